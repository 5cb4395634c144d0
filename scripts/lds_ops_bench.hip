// lds_ops_bench.hip -- LDS operation throughput on gfx950 (tuning evidence for
// the Bloom insert partition).  Standalone, not part of
// librsketch.  Every lane issues ITERS LDS operations at pseudo-random word
// addresses inside a table of `words` u32 (the shapes the partition kernels
// use: 18283-bin histograms, 256-bin rank counters, 16384-word slices).
//   hipcc -O3 --offload-arch=gfx950 -o build/lds_ops_bench scripts/lds_ops_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int ITERS = 1024;
constexpr int MAXW = 32768;

template <int OP>
__global__ __launch_bounds__(1024) void lds_kernel(uint32_t words, uint32_t* out) {
  __shared__ uint32_t t[MAXW];
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) t[i] = i;
  __syncthreads();
  uint32_t x = (blockIdx.x * 1024 + threadIdx.x) * 2654435761u + 12345u;
  uint32_t acc = 0;
  const uint32_t mask = words - 1;  // words is a power of two here except OP 5
#pragma unroll 8
  for (int it = 0; it < ITERS; ++it) {
    x = x * 1664525u + 1013904223u;
    const uint32_t a = (OP == 5) ? (x >> 8) % words : (x >> 8) & mask;
    if (OP == 0) atomicAdd(&t[a], 1u);                     // ds_add_u32 (no return)
    if (OP == 1) acc += atomicAdd(&t[a], 1u);              // ds_add_rtn_u32
    if (OP == 2) atomicOr(&t[a], 1u << (x & 31));           // ds_or_b32
    if (OP == 3) t[a] = x;                                  // ds_write_b32 (racy, timing only)
    if (OP == 4) acc += t[a];                               // ds_read_b32
    if (OP == 5) atomicAdd(&t[a], 1u);                     // ds_add_u32, non-power-of-two table
    if (OP == 6) acc += t[(threadIdx.x + it * 64) & mask];  // ds_read_b32 conflict-free
  }
  __syncthreads();
  if (OP == 1 || OP == 4 || OP == 6) out[blockIdx.x * 1024 + threadIdx.x] = acc;
  else if (threadIdx.x == 0) out[blockIdx.x] = t[blockIdx.x & mask];
}

template <int OP>
double run(uint32_t words, int blocks, uint32_t* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(lds_kernel<OP>, dim3(blocks), dim3(1024), 0, 0, words, out);
  CK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(lds_kernel<OP>, dim3(blocks), dim3(1024), 0, 0, words, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return (double)blocks * 1024 * ITERS * 5 / (ms / 1e3);
}

int main() {
  int blocks = 256 * 4;
  uint32_t* out;
  CK(hipMalloc(&out, (size_t)blocks * 1024 * 4));
  struct {
    int op;
    uint32_t words;
    const char* name;
  } cases[] = {{0, 16384, "ds_add_u32 random, 16384 words"},  {0, 256, "ds_add_u32 random, 256 words"},
               {5, 18283, "ds_add_u32 random, 18283 words"},  {1, 256, "ds_add_rtn_u32 random, 256 words"},
               {1, 16384, "ds_add_rtn_u32 random, 16384 words"}, {2, 16384, "ds_or_b32 random, 16384 words"},
               {3, 16384, "ds_write_b32 random, 16384 words"}, {4, 16384, "ds_read_b32 random, 16384 words"},
               {6, 16384, "ds_read_b32 conflict-free"}};
  printf("{\"blocks\": %d, \"threads\": 1024, \"ops_per_lane\": %d, \"results\": [\n", blocks, ITERS);
  for (size_t i = 0; i < sizeof(cases) / sizeof(cases[0]); ++i) {
    double r = 0;
    switch (cases[i].op) {
      case 0: r = run<0>(cases[i].words, blocks, out); break;
      case 1: r = run<1>(cases[i].words, blocks, out); break;
      case 2: r = run<2>(cases[i].words, blocks, out); break;
      case 3: r = run<3>(cases[i].words, blocks, out); break;
      case 4: r = run<4>(cases[i].words, blocks, out); break;
      case 5: r = run<5>(cases[i].words, blocks, out); break;
      case 6: r = run<6>(cases[i].words, blocks, out); break;
    }
    printf("  {\"op\": \"%s\", \"Gops_per_s\": %.1f, \"lane_ops_per_clk_per_CU_at_2.4GHz\": %.2f}%s\n",
           cases[i].name, r / 1e9, r / 256 / 2.4e9, i + 1 < sizeof(cases) / sizeof(cases[0]) ? "," : "");
  }
  printf("]}\n");
  return 0;
}
