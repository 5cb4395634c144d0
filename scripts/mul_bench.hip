// mul_bench.hip -- integer-multiply and MurmurHash64A throughput on gfx950
// (tuning evidence for the C4 variable-length PFADD).
// Standalone, not part of librsketch; all data in registers (no memory).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mul_bench scripts/mul_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

constexpr uint64_t M = 0xc6a4a7935bd1e995ULL;
constexpr int ITERS = 4096;

// 8 independent 64-bit multiply chains per lane (x *= M): 3 multiply instrs each.
__global__ __launch_bounds__(256) void mul64_kernel(uint64_t seed, uint64_t* out) {
  uint64_t x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i + blockIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] *= M;
  }
  uint64_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) a ^= x[i];
  if (a == 0x1234) out[0] = a;
}

// 8 chains of 32-bit v_mul_lo_u32.
__global__ __launch_bounds__(256) void mul32_kernel(uint32_t seed, uint32_t* out) {
  uint32_t x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i + blockIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] *= 0x5bd1e995u;
  }
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) a ^= x[i];
  if (a == 0x1234) out[0] = a;
}

// 8 chains of 24-bit v_mul_u32_u24 (full rate candidate).
__global__ __launch_bounds__(256) void mul24_kernel(uint32_t seed, uint32_t* out) {
  uint32_t x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i + blockIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __umul24(x[i] & 0xFFFFFF, 0x5bd1e9u) + x[i];
  }
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) a ^= x[i];
  if (a == 0x1234) out[0] = a;
}

// MurmurHash64A of register-resident keys, lengths 8..64 (mean 36), sorted
// per wave (lane-uniform length) or mixed.
__device__ __forceinline__ uint64_t mix(uint64_t k) {
  k *= M;
  k ^= k >> 47;
  k *= M;
  return k;
}
template <bool UNIFORM>
__global__ __launch_bounds__(256) void murmur_kernel(uint64_t seed, uint64_t* out, uint64_t keys_per_lane) {
  uint64_t acc = 0;
  uint64_t w = seed + threadIdx.x + blockIdx.x * 256;
  for (uint64_t q = 0; q < keys_per_lane; ++q) {
    const uint32_t len = UNIFORM ? 8 + ((q * 2654435761u) >> 7) % 57 : 8 + ((w * 2654435761u + q * 40503u) >> 9) % 57;
    uint64_t h = 0xadc83b19ULL ^ (len * M);
    const uint32_t nb = len >> 3;
    for (uint32_t j = 0; j < nb; ++j) {
      h ^= mix(w + j * 0x9E3779B97F4A7C15ULL);
      h *= M;
    }
    if (len & 7) {
      h ^= (w >> (len & 7));
      h *= M;
    }
    h ^= h >> 47;
    h *= M;
    h ^= h >> 47;
    acc += h;
    w += 0x632BE59BD9B4E019ULL;
  }
  if (acc == 0x1234) out[0] = acc;
}

template <class F>
double timed(F&& launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipEventRecord(a));
  for (int r = 0; r < 3; ++r) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / 3;
}

int main() {
  const int blocks = 256 * 8;
  uint64_t* o64;
  CK(hipMalloc(&o64, 64));
  const double lanes = (double)blocks * 256;
  double ms = timed([&] { hipLaunchKernelGGL(mul64_kernel, dim3(blocks), dim3(256), 0, 0, 1ull, o64); });
  printf("{\"mul64_Gops\": %.1f, ", lanes * ITERS * 8 / (ms / 1e3) / 1e9);
  ms = timed([&] { hipLaunchKernelGGL(mul32_kernel, dim3(blocks), dim3(256), 0, 0, 1u, (uint32_t*)o64); });
  printf("\"mul32_Gops\": %.1f, ", lanes * ITERS * 8 / (ms / 1e3) / 1e9);
  ms = timed([&] { hipLaunchKernelGGL(mul24_kernel, dim3(blocks), dim3(256), 0, 0, 1u, (uint32_t*)o64); });
  printf("\"mul24_Gops\": %.1f, ", lanes * ITERS * 8 / (ms / 1e3) / 1e9);
  const uint64_t kpl = 1000000000ull / (uint64_t)lanes + 1;
  ms = timed([&] { hipLaunchKernelGGL(murmur_kernel<true>, dim3(blocks), dim3(256), 0, 0, 1ull, o64, kpl); });
  printf("\"murmur_uniform_len_1e9_keys_ms\": %.3f, ", ms * 1e9 / (kpl * lanes));
  ms = timed([&] { hipLaunchKernelGGL(murmur_kernel<false>, dim3(blocks), dim3(256), 0, 0, 1ull, o64, kpl); });
  printf("\"murmur_mixed_len_1e9_keys_ms\": %.3f}\n", ms * 1e9 / (kpl * lanes));
  return 0;
}
