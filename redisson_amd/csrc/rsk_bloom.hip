// rsk_bloom.hip -- Bloom-filter kernels for gfx950.
//
// Replaces RedissonBloomFilter's client-side index generation
// (src/main/java/org/redisson/RedissonBloomFilter.java:116-131: xxHash64 r39
// + FarmHash-uo double hashing, idx_i = (h_i & Long.MAX_VALUE) % size) and the
// k SETBIT / GETBIT commands it pipelines to Redis (:94-98, :147-151), and
// BITCOUNT for count() (:188-199).
//
// Data layout in HBM: the filter is the Redis string itself -- ceil(size/8)
// bytes, bit i in byte i>>3 under mask 0x80>>(i&7) (bitops.c, MSB-first;
// RedissonBitSet.java:152-173) -- addressed as little-endian u32 words so a
// SETBIT is one memory-side atomicOr: word i>>5, bit 8*((i>>3)&3) + 7-(i&7).
// Bounded by random 4-byte accesses, not by streaming bandwidth.
#include <hipcub/hipcub.hpp>

#include "rsk_bloom_kern.h"
#include "rsk_internal.h"

namespace rsk {

RSK_DEV uint32_t bit_mask(uint64_t idx) { return bloom_bit_mask(idx); }

template <bool FIXED16>
RSK_DEV void key_hashes(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                        uint64_t i, uint64_t& h1, uint64_t& h2) {
  bloom_key_hashes<FIXED16>(data, offsets, fixed_len, i, h1, h2);
}

template <bool FIXED16>
__global__ __launch_bounds__(256) void bloom_add_kernel(const uint8_t* __restrict__ data,
                                                        const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                        uint64_t n, uint32_t* __restrict__ bits, FastMod63 fm,
                                                        int k) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h1, h2;
    key_hashes<FIXED16>(data, offsets, fixed_len, i, h1, h2);
    ProbeSeq ps(h1, h2, fm);
    for (int t = 0; t < k; ++t) {
      atomicOr(&bits[ps.idx >> 5], bit_mask(ps.idx));
      if (t + 1 < k) ps.next(t, fm);
    }
  }
}

static uint32_t grid_for(rsk_ctx* c, uint64_t n);

template <int U>
static void launch_contains_ee(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out, uint32_t blocks_per_cu) {
  uint64_t g = (k.n + 256 * U - 1) / (256 * U);
  uint64_t cap = (uint64_t)c->num_cus * blocks_per_cu;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  hipLaunchKernelGGL(bloom_contains16_ee_kernel<U>, dim3((uint32_t)g), dim3(256), 0, c->stream,
                     reinterpret_cast<const uint4*>(k.data), k.n, b->d_bits, b->fm, b->k, d_out);
}

static bool fixed16(const DevKeys& k) {
  return k.offsets == nullptr && k.fixed_len == 16 && (reinterpret_cast<uintptr_t>(k.data) & 15) == 0;
}
static uint32_t grid_for(rsk_ctx* c, uint64_t n) {
  uint64_t g = (n + 255) / 256;
  uint64_t cap = (uint64_t)c->num_cus * 32;
  return (uint32_t)(g < cap ? (g ? g : 1) : cap);
}

// k random memory-side atomicOr per key (small batches).
void bloom_add_direct_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k) {
  if (k.n == 0) return;
  if (fixed16(k))
    hipLaunchKernelGGL(bloom_add_kernel<true>, dim3(grid_for(c, k.n)), dim3(256), 0, c->stream, k.data, nullptr, 16u,
                       k.n, b->d_bits, b->fm, b->k);
  else
    hipLaunchKernelGGL(bloom_add_kernel<false>, dim3(grid_for(c, k.n)), dim3(256), 0, c->stream, k.data, k.offsets,
                       k.fixed_len, k.n, b->d_bits, b->fm, b->k);
  RSK_CHECK_LAUNCH("bloom_add_direct");
}

// Large batches: probes routed to LDS-resident 64 KiB filter slices, by the
// super-tile partition (rsk_bloom_st.hip; k <= 16) or the exact-offset
// pipeline (rsk_bloom_part.hip); small ones: direct atomics.
void bloom_add_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k) {
  if (k.n == 0) return;
  ProfScope ps(c, fixed16(k) ? "bloom_add16" : "bloom_add");
  if (bloom_add_supertile(c, b, k)) return;
  if (bloom_add_partitioned(c, b, k)) return;
  bloom_add_direct_launch(c, b, k);
}

void bloom_contains_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out) {
  if (k.n == 0) return;
  if (fixed16(k)) {
    ProfScope ps(c, "bloom_contains16");
    launch_contains_ee<2>(c, b, k, d_out, 32);
    RSK_CHECK_LAUNCH("bloom_contains16");
  } else {
    ProfScope ps(c, "bloom_contains");
    hipLaunchKernelGGL(bloom_contains_kernel<false>, dim3(grid_for(c, k.n)), dim3(256), 0, c->stream, k.data,
                       k.offsets, k.fixed_len, k.n, b->d_bits, b->fm, b->k, d_out);
    RSK_CHECK_LAUNCH("bloom_contains");
  }
}

// ------------------------------------------- add() replies, input order
// Probe p = i*k + t.  A probe "finds its bit clear" iff the bit was clear
// before the batch and p is the first probe (in sequence order) of that
// bit.  Stable radix sort of (bit index, p) finds the first probe per bit.
__global__ void bloom_probe_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                                   uint32_t fixed_len, uint64_t n, const uint32_t* __restrict__ bits, FastMod63 fm,
                                   int k, uint64_t* __restrict__ pidx, uint32_t* __restrict__ pseq,
                                   uint8_t* __restrict__ pclear) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h1, h2;
    key_hashes<false>(data, offsets, fixed_len, i, h1, h2);
    ProbeSeq ps(h1, h2, fm);
    for (int t = 0; t < k; ++t) {
      const uint64_t idx = ps.idx;
      if (t + 1 < k) ps.next(t, fm);
      uint64_t p = i * (uint64_t)k + t;
      pidx[p] = idx;
      pseq[p] = (uint32_t)p;
      pclear[p] = (bits[idx >> 5] & bit_mask(idx)) == 0;
    }
  }
}

__global__ void bloom_first_kernel(const uint64_t* __restrict__ sidx, const uint32_t* __restrict__ sseq, uint64_t np,
                                   const uint8_t* __restrict__ pclear, uint8_t* __restrict__ found0) {
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < np; q += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t p = sseq[q];
    bool first = q == 0 || sidx[q] != sidx[q - 1];
    found0[p] = first && pclear[p];
  }
}

__global__ void bloom_reply_kernel(const uint8_t* __restrict__ found0, uint64_t n, int k, uint8_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t r = 0;
    for (int t = 0; t < k - 1; ++t) r |= found0[i * k + t];
    out[i] = r;
  }
}

void bloom_add_each_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out) {
  const uint64_t n = k.n;
  if (n == 0) return;
  const uint64_t np = n * (uint64_t)b->k;
  int end_bit = 1;
  while (end_bit < 64 && ((uint64_t)(b->size - 1) >> end_bit) != 0) ++end_bit;
  size_t tmp_bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                     (uint32_t*)nullptr, (int)np, 0, end_bit, c->stream);
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  uint64_t need = 2 * al(np * 8) + 2 * al(np * 4) + 2 * al(np) + al(tmp_bytes);
  uint8_t* w = c->work(need);
  uint64_t* idx_in = reinterpret_cast<uint64_t*>(w);
  uint64_t* idx_out = reinterpret_cast<uint64_t*>(w + al(np * 8));
  uint32_t* seq_in = reinterpret_cast<uint32_t*>(w + 2 * al(np * 8));
  uint32_t* seq_out = reinterpret_cast<uint32_t*>(w + 2 * al(np * 8) + al(np * 4));
  uint8_t* pclear = w + 2 * al(np * 8) + 2 * al(np * 4);
  uint8_t* found0 = pclear + al(np);
  void* tmp = found0 + al(np);
  ProfScope ps(c, "bloom_add_each");
  hipLaunchKernelGGL(bloom_probe_kernel, dim3(grid_for(c, n)), dim3(256), 0, c->stream, k.data, k.offsets, k.fixed_len,
                     n, b->d_bits, b->fm, b->k, idx_in, seq_in, pclear);
  RSK_CHECK_LAUNCH("bloom_probe");
  RSK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, idx_in, idx_out, seq_in, seq_out, (int)np, 0, end_bit,
                                             c->stream));
  hipLaunchKernelGGL(bloom_first_kernel, dim3(grid_for(c, np)), dim3(256), 0, c->stream, idx_out, seq_out, np, pclear,
                     found0);
  RSK_CHECK_LAUNCH("bloom_first");
  hipLaunchKernelGGL(bloom_reply_kernel, dim3(grid_for(c, n)), dim3(256), 0, c->stream, found0, n, b->k, d_out);
  RSK_CHECK_LAUNCH("bloom_reply");
  bloom_add_launch(c, b, k);
}

// The sort path bounded for its 32-bit sort: sub-batches of <= 2^28 probes,
// each answered against the filter the previous ones left.
void bloom_add_replies_sorted(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out) {
  const uint64_t max_keys = std::max<uint64_t>(1, (1ull << 28) / (uint64_t)b->k);
  for (uint64_t done = 0; done < k.n; done += max_keys) {
    DevKeys sub = k;
    sub.n = std::min<uint64_t>(max_keys, k.n - done);
    if (k.offsets) sub.offsets = k.offsets + done;
    else sub.data = k.data + done * k.fixed_len;
    bloom_add_each_launch(c, b, sub, d_out + done);
  }
}

void bloom_add_replies_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out) {
  if (k.n == 0) return;
  if (bloom_add_replies_append(c, b, k, d_out)) return;
  bloom_add_replies_sorted(c, b, k, d_out);
}

// BITCOUNT over the filter words.
__global__ __launch_bounds__(256) void popcount_kernel(const uint32_t* __restrict__ w, uint64_t nwords,
                                                       unsigned long long* __restrict__ out) {
  uint64_t acc = 0;
  const uint64_t n4 = nwords / 4;
  const uint4* w4 = reinterpret_cast<const uint4*>(w);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = ld_nt16(&w4[i]);
    acc += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
  }
  for (uint64_t i = n4 * 4 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords;
       i += (uint64_t)gridDim.x * blockDim.x)
    acc += __popc(w[i]);
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  __shared__ uint64_t part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(part[0] + part[1] + part[2] + part[3]));
}

void bloom_bitcount_launch(rsk_ctx* c, const uint32_t* d_bits, uint64_t nwords, uint64_t* d_out) {
  RSK_HIP(hipMemsetAsync(d_out, 0, 8, c->stream));
  uint64_t g = (nwords / 4 + 255) / 256;
  uint64_t cap = (uint64_t)c->num_cus * 8;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  ProfScope ps(c, "bitcount");
  hipLaunchKernelGGL(popcount_kernel, dim3((uint32_t)g), dim3(256), 0, c->stream, d_bits, nwords,
                     reinterpret_cast<unsigned long long*>(d_out));
  RSK_CHECK_LAUNCH("bitcount");
}

// bits |= src (byte string of nbytes), the receive side of a slice-OR merge.
__global__ __launch_bounds__(256) void or_bytes_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                       uint64_t nbytes) {
  const uint64_t n16 = nbytes / 16;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 a = reinterpret_cast<uint4*>(dst)[i];
    uint4 b;
    __builtin_memcpy(&b, src + 16 * i, 16);
    reinterpret_cast<uint4*>(dst)[i] = make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w);
  }
  for (uint64_t i = n16 * 16 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes;
       i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] |= src[i];
}

void bloom_or_launch(rsk_ctx* c, uint32_t* d_bits, const uint8_t* d_src, uint64_t nbytes) {
  uint64_t g = (nbytes / 16 + 255) / 256;
  uint64_t cap = (uint64_t)c->num_cus * 8;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  ProfScope ps(c, "bloom_or");
  hipLaunchKernelGGL(or_bytes_kernel, dim3((uint32_t)g), dim3(256), 0, c->stream, reinterpret_cast<uint8_t*>(d_bits),
                     d_src, nbytes);
  RSK_CHECK_LAUNCH("bloom_or");
}

// dst |= OR of the rows (the local step of the slice-OR merge): 16-byte
// lanes over the aligned body, one word per lane over the tail.
__global__ __launch_bounds__(256) void or_rows_into_kernel(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                           uint32_t rows, uint64_t words, uint64_t stride) {
  const uint64_t w4 = words / 4;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = t0; i < w4; i += step) {
    uint4 acc = reinterpret_cast<const uint4*>(dst)[i];
    for (uint32_t r = 0; r < rows; ++r) {
      const uint4 v = reinterpret_cast<const uint4*>(src + (uint64_t)r * stride)[i];
      acc = make_uint4(acc.x | v.x, acc.y | v.y, acc.z | v.z, acc.w | v.w);
    }
    reinterpret_cast<uint4*>(dst)[i] = acc;
  }
  for (uint64_t i = 4 * w4 + t0; i < words; i += step) {
    uint32_t acc = dst[i];
    for (uint32_t r = 0; r < rows; ++r) acc |= src[(uint64_t)r * stride + i];
    dst[i] = acc;
  }
}

void or_rows_into_launch(rsk_ctx* c, uint32_t* d_dst, const uint32_t* d_src, uint32_t rows, uint64_t words,
                         uint64_t stride) {
  uint64_t g = (words / 4 + 255) / 256;
  const uint64_t cap = (uint64_t)c->num_cus * 8;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  ProfScope ps(c, "bloom_or_rows");
  hipLaunchKernelGGL(or_rows_into_kernel, dim3((uint32_t)g), dim3(256), 0, c->stream, d_dst, d_src, rows, words,
                     stride);
  RSK_CHECK_LAUNCH("bloom_or_rows");
}

}  // namespace rsk

namespace rsk {

// ------------------------------------------------ misc/Hash.hashToBase64
// src/main/java/org/redisson/misc/Hash.java:29-40: h1 = farmUo(bytes),
// h2 = xx_r39(bytes), written as two big-endian longs (ByteBuf.writeLong),
// standard Base64 with padding, the trailing "==" dropped: 22 characters per
// key (RedissonMultimap.java:62 and RedissonCache.java:160 name keys by it).
__global__ __launch_bounds__(256) void hash_b64_kernel(const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                       uint64_t n, char* __restrict__ out) {
  const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h1, h2;  // bloom_key_hashes gives (xx, farm); Hash.java writes farm first
    bloom_key_hashes<false>(data, offsets, fixed_len, i, h2, h1);
    uint8_t b[18];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      b[q] = (uint8_t)(h1 >> (56 - 8 * q));
      b[8 + q] = (uint8_t)(h2 >> (56 - 8 * q));
    }
    b[16] = b[17] = 0;
    char* o = out + 22 * i;
#pragma unroll
    for (int g = 0; g < 6; ++g) {  // 6 groups of 3 bytes -> 24 chars; the last 2 ('=' padding) dropped
      const uint32_t v = ((uint32_t)b[3 * g] << 16) | ((uint32_t)b[3 * g + 1] << 8) | b[3 * g + 2];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (4 * g + c < 22) o[4 * g + c] = A[(v >> (18 - 6 * c)) & 63];
    }
  }
}

void hash_b64_launch(rsk_ctx* c, const DevKeys& k, char* d_out) {
  if (k.n == 0) return;
  uint64_t g = (k.n + 255) / 256;
  const uint64_t cap = (uint64_t)c->num_cus * 16;
  if (g > cap) g = cap;
  ProfScope ps(c, "hash_b64");
  hipLaunchKernelGGL(hash_b64_kernel, dim3((uint32_t)g), dim3(256), 0, c->stream, k.data, k.offsets, k.fixed_len, k.n,
                     d_out);
  RSK_CHECK_LAUNCH("hash_b64");
}

}  // namespace rsk
