// rsk_gen.hip -- on-device synthetic key streams, so that the
// benchmark inputs are resident in HBM before the timed region.  The same
// streams are restated on the CPU in oracle/rsk_oracle.c (orc_gen_*).
#include <cmath>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "rsk_diag_internal.h"

namespace rsk {

// C2: key i = (splitmix64(s+2i), splitmix64(s+2i+1)) little-endian.
__global__ void gen_keys16_kernel(uint64_t seed, uint64_t start, uint64_t n, uint4* __restrict__ out) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i = start + j;
    uint64_t lo = splitmix64(seed + 2 * i), hi = splitmix64(seed + 2 * i + 1);
    out[j] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
}

// C5: group = splitmix64(s+3i) mod G, key = (splitmix64(s+3i+1), splitmix64(s+3i+2)).
__global__ void gen_grouped_kernel(uint64_t seed, uint64_t G, uint64_t start, uint64_t n, uint32_t* __restrict__ groups,
                                   uint4* __restrict__ keys) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i = start + j;
    groups[j] = (uint32_t)(splitmix64(seed + 3 * i) % G);
    uint64_t lo = splitmix64(seed + 3 * i + 1), hi = splitmix64(seed + 3 * i + 2);
    keys[j] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
}

// C5 Zipf(s) stress variant: as gen_grouped_kernel, but the
// group is the Zipf rank of u = splitmix64(s+3i) >> 1: the first r with
// u < cdf[r] (cdf: u63 fixed-point cumulative weights r^-s, built on the host
// by zipf_cdf below and restated in oracle/rsk_oracle.c orc_zipf_cdf).
__global__ void gen_grouped_zipf_kernel(uint64_t seed, const uint64_t* __restrict__ cdf, uint32_t G, uint64_t start,
                                        uint64_t n, uint32_t* __restrict__ groups, uint4* __restrict__ keys) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i = start + j;
    const uint64_t u = splitmix64(seed + 3 * i) >> 1;
    uint32_t lo = 0, hi = G - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (u < cdf[mid]) hi = mid;
      else lo = mid + 1;
    }
    groups[j] = lo;
    uint64_t a = splitmix64(seed + 3 * i + 1), b = splitmix64(seed + 3 * i + 2);
    keys[j] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
  }
}

// C3 queries: r = splitmix64(q+3j); r&1 -> inserted key (r>>1) mod n_ins,
// else fresh (splitmix64(q+3j+1), splitmix64(q+3j+2)).
constexpr uint64_t FRESH_TAG = 1ULL << 63;

__global__ void gen_queries16_kernel(uint64_t qseed, uint64_t iseed, uint64_t n_ins, uint64_t start, uint64_t n,
                                     uint4* __restrict__ out) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t q = start + j;
    uint64_t r = splitmix64(qseed + 3 * q);
    uint64_t lo, hi;
    if (r & 1) {
      uint64_t i = (r >> 1) % n_ins;
      lo = splitmix64(iseed + 2 * i);
      hi = splitmix64(iseed + 2 * i + 1);
    } else {
      // bit 63 set: a state range the insert stream (iseed + j, j < 2^62)
      // never reaches, so a fresh key is never an inserted one
      lo = splitmix64((qseed + 3 * q + 1) | FRESH_TAG);
      hi = splitmix64((qseed + 3 * q + 2) | FRESH_TAG);
    }
    out[j] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
}

// C4: len_i = 8 + splitmix64(s ^ i) mod 57, bytes 0x21 + (b mod 94) with b
// the bytes of splitmix64(s + 8i + w).  Lengths are written to offs[j+1];
// the caller scans them into offsets.
__global__ void gen_varlen_len_kernel(uint64_t seed, uint64_t start, uint64_t n, uint64_t* __restrict__ offs) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    offs[j + 1] = 8 + splitmix64(seed ^ (start + j)) % 57;
  }
}

__global__ void gen_varlen_bytes_kernel(uint64_t seed, uint64_t start, uint64_t n, const uint64_t* __restrict__ offs,
                                        uint8_t* __restrict__ blob) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i = start + j;
    uint64_t s = offs[j], len = offs[j + 1] - s;
    for (uint32_t w = 0; w * 8 < len; ++w) {
      uint64_t r = splitmix64(seed + (i << 3) + w);
      for (uint32_t b = 0; b < 8 && w * 8 + b < len; ++b)
        blob[s + w * 8 + b] = (uint8_t)(0x21 + ((r >> (8 * b)) & 0xFF) % 94);
    }
  }
}

static uint32_t gen_grid(rsk_ctx* c, uint64_t n) {
  uint64_t g = (n + 255) / 256;
  uint64_t cap = (uint64_t)c->num_cus * 16;
  return (uint32_t)(g < cap ? (g ? g : 1) : cap);
}

void gen_keys16_launch(rsk_ctx* c, uint64_t seed, uint64_t start, uint64_t n, void* out) {
  hipLaunchKernelGGL(gen_keys16_kernel, dim3(gen_grid(c, n)), dim3(256), 0, c->stream, seed, start, n,
                     reinterpret_cast<uint4*>(out));
  RSK_CHECK_LAUNCH("gen_keys16");
}

void gen_grouped_launch(rsk_ctx* c, uint64_t seed, uint64_t G, uint64_t start, uint64_t n, uint32_t* g, void* keys) {
  hipLaunchKernelGGL(gen_grouped_kernel, dim3(gen_grid(c, n)), dim3(256), 0, c->stream, seed, G, start, n, g,
                     reinterpret_cast<uint4*>(keys));
  RSK_CHECK_LAUNCH("gen_grouped");
}

// cdf[r] = floor(2^63 * sum_{q<=r+1} q^-s / sum_{q<=G} q^-s), cdf[G-1] = 2^63
// (every u < 2^63 lands): two sequential double passes, glibc pow.
std::vector<uint64_t> zipf_cdf(uint32_t G, double s) {
  double total = 0.0;
  for (uint32_t r = 1; r <= G; ++r) total += std::pow((double)r, -s);
  std::vector<uint64_t> cdf(G);
  double cum = 0.0;
  for (uint32_t r = 1; r <= G; ++r) {
    cum += std::pow((double)r, -s);
    cdf[r - 1] = (uint64_t)std::ldexp(cum / total, 63);
  }
  cdf[G - 1] = 1ull << 63;
  return cdf;
}

void gen_grouped_zipf_launch(rsk_ctx* c, uint64_t seed, const uint64_t* d_cdf, uint32_t G, uint64_t start, uint64_t n,
                             uint32_t* g, void* keys) {
  hipLaunchKernelGGL(gen_grouped_zipf_kernel, dim3(gen_grid(c, n)), dim3(256), 0, c->stream, seed, d_cdf, G, start, n,
                     g, reinterpret_cast<uint4*>(keys));
  RSK_CHECK_LAUNCH("gen_grouped_zipf");
}

void gen_queries16_launch(rsk_ctx* c, uint64_t qseed, uint64_t iseed, uint64_t n_ins, uint64_t start, uint64_t n,
                          void* out) {
  hipLaunchKernelGGL(gen_queries16_kernel, dim3(gen_grid(c, n)), dim3(256), 0, c->stream, qseed, iseed, n_ins, start,
                     n, reinterpret_cast<uint4*>(out));
  RSK_CHECK_LAUNCH("gen_queries16");
}

void gen_varlen_lengths_launch(rsk_ctx* c, uint64_t seed, uint64_t start, uint64_t n, uint64_t* offsets) {
  RSK_HIP(hipMemsetAsync(offsets, 0, 8, c->stream));
  hipLaunchKernelGGL(gen_varlen_len_kernel, dim3(gen_grid(c, n)), dim3(256), 0, c->stream, seed, start, n, offsets);
  RSK_CHECK_LAUNCH("gen_varlen_len");
  // Inclusive scan of offsets[1..n] in place (offsets[0] = 0).
  size_t tmp_bytes = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, offsets + 1, offsets + 1, (int)n, c->stream);
  void* tmp = nullptr;  // the support library keeps no scratch of its own
  RSK_HIP(hipMalloc(&tmp, tmp_bytes + 256));
  hipError_t e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, offsets + 1, offsets + 1, (int)n, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(tmp);
  RSK_HIP(e);
}

void gen_varlen_bytes_launch(rsk_ctx* c, uint64_t seed, uint64_t start, uint64_t n, const uint64_t* offsets,
                             uint8_t* blob) {
  hipLaunchKernelGGL(gen_varlen_bytes_kernel, dim3(gen_grid(c, n)), dim3(256), 0, c->stream, seed, start, n, offsets,
                     blob);
  RSK_CHECK_LAUNCH("gen_varlen_bytes");
}

}  // namespace rsk

using namespace rsk;

extern "C" {

// ----------------------------------------------------------- generators
int rsk_gen_keys16(rsk_ctx* c, uint64_t seed, uint64_t start, uint64_t n, void* dev_out) {
  return diag::guarded([&] {
    diag::need(c && (dev_out || n == 0), "NULL argument");
    diag::Lock l(c);
    if (n) gen_keys16_launch(c, seed, start, n, dev_out);
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_gen_grouped(rsk_ctx* c, uint64_t seed, uint64_t G, uint64_t start, uint64_t n, uint32_t* dev_groups,
                    void* dev_keys) {
  return diag::guarded([&] {
    diag::need(c && G > 0 && ((dev_groups && dev_keys) || n == 0), "bad arguments");
    diag::Lock l(c);
    if (n) gen_grouped_launch(c, seed, G, start, n, dev_groups, dev_keys);
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_gen_grouped_zipf(rsk_ctx* c, uint64_t seed, uint64_t G, double s, uint64_t start, uint64_t n,
                         uint32_t* dev_groups, void* dev_keys) {
  return diag::guarded([&] {
    diag::need(c && G > 0 && G < (1ull << 32) && ((dev_groups && dev_keys) || n == 0), "bad arguments");
    diag::need(s > 0.0 && s < 16.0, "Zipf exponent must be in (0, 16)");
    diag::Lock l(c);
    if (!n) return;
    const std::vector<uint64_t> cdf = zipf_cdf((uint32_t)G, s);
    uint64_t* d_cdf = nullptr;
    RSK_HIP(hipMalloc(&d_cdf, 8 * G));
    hipError_t e = hipMemcpyAsync(d_cdf, cdf.data(), 8 * G, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
      gen_grouped_zipf_launch(c, seed, d_cdf, (uint32_t)G, start, n, dev_groups, dev_keys);
      e = hipStreamSynchronize(c->stream);
    }
    (void)hipFree(d_cdf);
    RSK_HIP(e);
  });
}

int rsk_gen_queries16(rsk_ctx* c, uint64_t qseed, uint64_t iseed, uint64_t n_ins, uint64_t start, uint64_t n,
                      void* dev_out) {
  return diag::guarded([&] {
    diag::need(c && n_ins > 0 && (dev_out || n == 0), "bad arguments");
    diag::Lock l(c);
    if (n) gen_queries16_launch(c, qseed, iseed, n_ins, start, n, dev_out);
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_gen_varlen(rsk_ctx* c, uint64_t seed, uint64_t start, uint64_t n, uint64_t* dev_offsets, void* dev_blob,
                   uint64_t blob_cap, uint64_t* total_bytes) {
  return diag::guarded([&] {
    diag::need(c && dev_offsets && total_bytes, "NULL argument");
    diag::need(n < (1ull << 31), "n must be < 2^31 per call");
    diag::Lock l(c);
    gen_varlen_lengths_launch(c, seed, start, n, dev_offsets);
    uint64_t tot = 0;
    RSK_HIP(hipMemcpyAsync(&tot, dev_offsets + n, 8, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    *total_bytes = tot;
    if (dev_blob) {
      diag::need(blob_cap >= tot, "blob capacity too small");
      gen_varlen_bytes_launch(c, seed, start, n, dev_offsets, reinterpret_cast<uint8_t*>(dev_blob));
      RSK_HIP(hipStreamSynchronize(c->stream));
    }
  });
}

}  // extern "C"
