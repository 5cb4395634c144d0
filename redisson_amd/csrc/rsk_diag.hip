// rsk_diag.hip -- memory-system microbenchmarks that give the sketch kernels
// their measured roofline denominators on the box they run on:
//   mode 0: streaming read (16 B/lane nontemporal loads)  -> GB/s
//   mode 1: random 4 B gathers over the buffer            -> gathers/s
//   mode 2: random 4 B atomicOr over the buffer           -> atomics/s
//   mode 3: streaming copy (read + write halves)          -> GB/s (read+write)
// Indices come from splitmix64(i), as uniform as the Bloom probe stream.
#include <cstring>

#include "rsk_internal.h"

namespace rsk {

__global__ __launch_bounds__(256) void diag_stream_read(const uint4* __restrict__ p, uint64_t n16,
                                                        uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = ld_nt16(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads alive
}

__global__ __launch_bounds__(256) void diag_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = ld_nt16(src + i);
}

__global__ __launch_bounds__(256) void diag_gather(const uint32_t* __restrict__ w, uint64_t nwords, uint64_t nops,
                                                   uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nops; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t r = splitmix64(i);
    acc ^= w[__umul64hi(r, nwords)];
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void diag_atomic_or(uint32_t* __restrict__ w, uint64_t nwords, uint64_t nops) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nops; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t r = splitmix64(i);
    atomicOr(&w[__umul64hi(r, nwords)], 1u << (r & 31));
  }
}

}  // namespace rsk

extern "C" int rsk_diag_hll_variant(rsk_ctx* c, int variant, const void* dev_keys16, uint64_t n, double* ms) {
  try {
    if (!c || !dev_keys16 || !ms || n == 0) throw rsk::RskError{RSK_ERR_INVALID_ARG, "bad arguments"};
    std::lock_guard<std::recursive_mutex> g(c->mu);
    RSK_HIP(hipSetDevice(c->device));
    hipEvent_t a, b;
    RSK_HIP(hipEventCreate(&a));
    RSK_HIP(hipEventCreate(&b));
    RSK_HIP(hipEventRecord(a, c->stream));
    rsk::hll_variant_launch(c, variant, reinterpret_cast<const uint4*>(dev_keys16), n);
    RSK_HIP(hipEventRecord(b, c->stream));
    RSK_HIP(hipEventSynchronize(b));
    float f = 0;
    RSK_HIP(hipEventElapsedTime(&f, a, b));
    *ms = f;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    rsk::set_error("");
    return RSK_OK;
  } catch (const rsk::RskError& e) {
    rsk::set_error(e.msg);
    return e.code;
  }
}

extern "C" int rsk_diag_bloom_contains_variant(rsk_ctx* c, int variant, rsk_bloom* bf, const void* dev_keys16,
                                               uint64_t n, uint8_t* dev_out, double* ms) {
  try {
    if (!c || !bf || !dev_keys16 || !dev_out || !ms || n == 0) throw rsk::RskError{RSK_ERR_INVALID_ARG, "bad arguments"};
    std::lock_guard<std::recursive_mutex> g(c->mu);
    RSK_HIP(hipSetDevice(c->device));
    hipEvent_t a, b;
    RSK_HIP(hipEventCreate(&a));
    RSK_HIP(hipEventCreate(&b));
    RSK_HIP(hipEventRecord(a, c->stream));
    rsk::bloom_contains_variant_launch(c, bf, rsk::DevKeys{reinterpret_cast<const uint8_t*>(dev_keys16), nullptr, n, 16},
                                       dev_out, variant);
    RSK_HIP(hipEventRecord(b, c->stream));
    RSK_HIP(hipEventSynchronize(b));
    float f = 0;
    RSK_HIP(hipEventElapsedTime(&f, a, b));
    *ms = f;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    rsk::set_error("");
    return RSK_OK;
  } catch (const rsk::RskError& e) {
    rsk::set_error(e.msg);
    return e.code;
  }
}

namespace rsk {
int bloom_occupancy_probe(int which, int* per_cu);
}
// Occupancy query result (hipError, per-CU workgroups) for the persistent
// Bloom kernels: which 0 = sa1 (512 lanes), 1 = the append apply.
extern "C" int rsk_diag_occupancy(int which, int* per_cu, int* hip_error) {
  *hip_error = rsk::bloom_occupancy_probe(which, per_cu);
  return RSK_OK;
}

extern "C" int rsk_diag_membench(rsk_ctx* c, int mode, void* buf, uint64_t bytes, uint64_t nops, double* ms) {
  try {
    if (!c || !buf || !ms || bytes < 64 || mode < 0 || mode > 3) throw rsk::RskError{RSK_ERR_INVALID_ARG, "bad arguments"};
    std::lock_guard<std::recursive_mutex> g(c->mu);
    RSK_HIP(hipSetDevice(c->device));
    hipEvent_t a, b;
    RSK_HIP(hipEventCreate(&a));
    RSK_HIP(hipEventCreate(&b));
    uint32_t* sink = reinterpret_cast<uint32_t*>(c->d_small + 512);
    const uint32_t grid = (uint32_t)c->num_cus * 8;
    RSK_HIP(hipEventRecord(a, c->stream));
    switch (mode) {
      case 0:
        hipLaunchKernelGGL(rsk::diag_stream_read, dim3(grid), dim3(256), 0, c->stream,
                           reinterpret_cast<const uint4*>(buf), bytes / 16, sink);
        break;
      case 1:
        hipLaunchKernelGGL(rsk::diag_gather, dim3(grid), dim3(256), 0, c->stream,
                           reinterpret_cast<const uint32_t*>(buf), bytes / 4, nops, sink);
        break;
      case 2:
        hipLaunchKernelGGL(rsk::diag_atomic_or, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<uint32_t*>(buf),
                           bytes / 4, nops);
        break;
      case 3: {
        const uint64_t half = bytes / 32;  // uint4 elements per half
        hipLaunchKernelGGL(rsk::diag_copy, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<const uint4*>(buf),
                           reinterpret_cast<uint4*>(buf) + half, half);
        break;
      }
    }
    RSK_CHECK_LAUNCH("diag");
    RSK_HIP(hipEventRecord(b, c->stream));
    RSK_HIP(hipEventSynchronize(b));
    float f = 0;
    RSK_HIP(hipEventElapsedTime(&f, a, b));
    *ms = f;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    rsk::set_error("");
    return RSK_OK;
  } catch (const rsk::RskError& e) {
    rsk::set_error(e.msg);
    return e.code;
  }
}

extern "C" int rsk_diag_bloom_contains_probes(rsk_ctx* c, rsk_bloom* bf, const void* dev_keys16, uint64_t n,
                                              uint8_t* dev_out, uint64_t* probes) {
  try {
    if (!c || !bf || !dev_keys16 || !dev_out || !probes || n == 0)
      throw rsk::RskError{RSK_ERR_INVALID_ARG, "bad arguments"};
    std::lock_guard<std::recursive_mutex> g(c->mu);
    RSK_HIP(hipSetDevice(c->device));
    auto* d = reinterpret_cast<unsigned long long*>(c->d_small + 384);
    RSK_HIP(hipMemsetAsync(d, 0, 8, c->stream));
    rsk::bloom_contains_probe_count_launch(
        c, bf, rsk::DevKeys{reinterpret_cast<const uint8_t*>(dev_keys16), nullptr, n, 16}, dev_out, d);
    RSK_HIP(hipMemcpyAsync(c->h_small + 384, d, 8, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(probes, c->h_small + 384, 8);
    rsk::set_error("");
    return RSK_OK;
  } catch (const rsk::RskError& e) {
    rsk::set_error(e.msg);
    return e.code;
  }
}

extern "C" int rsk_diag_hll_var_variant(rsk_ctx* c, int variant, const void* dev_data, const uint64_t* dev_offsets,
                                        uint64_t n, double* ms) {
  try {
    if (!c || !dev_data || !dev_offsets || !ms || n == 0) throw rsk::RskError{RSK_ERR_INVALID_ARG, "bad arguments"};
    std::lock_guard<std::recursive_mutex> g(c->mu);
    RSK_HIP(hipSetDevice(c->device));
    hipEvent_t a, b;
    RSK_HIP(hipEventCreate(&a));
    RSK_HIP(hipEventCreate(&b));
    RSK_HIP(hipEventRecord(a, c->stream));
    rsk::hll_var_variant_launch(c, variant, reinterpret_cast<const uint8_t*>(dev_data), dev_offsets, n);
    RSK_HIP(hipEventRecord(b, c->stream));
    RSK_HIP(hipEventSynchronize(b));
    float f = 0;
    RSK_HIP(hipEventElapsedTime(&f, a, b));
    *ms = f;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    rsk::set_error("");
    return RSK_OK;
  } catch (const rsk::RskError& e) {
    rsk::set_error(e.msg);
    return e.code;
  }
}
