// bloom_chain_bench.hip -- the C3 insert's per-key arithmetic alone, in
// registers (no memory): what the sa1 pass spends on the two hashes and the
// k probe indices (tuning evidence).
// Standalone, not part of librsketch.
//   hipcc -O3 --offload-arch=gfx950 -I redisson_amd/csrc -o /tmp/bcb scripts/bloom_chain_bench.hip
//   /tmp/bcb [size]     (default: C3's filter, 1e9 keys at 1 % -> 9585058378 bits; k = 7)
// Modes (1e9 keys each, ms from HIP events, median of 3):
//   0 key words only           1 + xxh64_16 + farm_16
//   2 + the round-4 probe sequence (fastmod63 twice, two corrections per step)
//   3 + rsk::ProbeSeq (the library: fastmod63 twice, one correction per step)
//   4 + rsk::ProbeSeq's step with fastmod63_big below (three 32-bit
//     multiplies per mod instead of seven; measured no faster, not adopted)
// and a check that forms 2, 3 and 4 give the same k indices for every key, and
// fastmod63 / fastmod63_big the same remainders at boundary dividends
// (multiples of d and their neighbours, 2^63 - 1 and below).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "rsk_device.h"

#define CK(x)                                                \
  do {                                                       \
    hipError_t e = (x);                                      \
    if (e != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                               \
    }                                                        \
  } while (0)

using namespace rsk;

static FastMod63 host_fastmod(uint64_t d) {
  FastMod63 f{};
  f.d = d;
  uint32_t l = 0;
  while (l < 64 && ((unsigned __int128)1 << l) < d) ++l;
  f.l = l;
  f.M = l ? (uint64_t)((((unsigned __int128)1 << (63 + l)) + d - 1) / d) : 0;
  f.r63 = (uint64_t)((1ULL << 63) % d);
  return f;
}

// The remainder for d > 2^32 (l >= 33) from the top 32 bits of x and of M:
// with x = xh 2^31 + xl and M = Mh 2^32 + Ml the dropped terms of x M are
// below 2^96 <= 2^(63+l), so (xh Mh) >> l is floor(x/d) or one less and
// x - q d lies in [0, 2d) (tests/test_probe_math.py restates it).
__device__ uint64_t fastmod63_big(uint64_t x, const FastMod63& f) {
  if (f.l < 33) return fastmod63(x, f);
  const uint64_t p = (uint64_t)(uint32_t)(x >> 31) * (uint32_t)(f.M >> 32);
  const uint32_t q = (uint32_t)(p >> f.l);
  const uint64_t r = x - (uint64_t)q * f.d;
  return r >= f.d ? r - f.d : r;
}

// The round-4 probe sequence (for the A/B only).
struct ProbeSeq4 {
  uint64_t v = 0, idx = 0, v1 = 0, v2 = 0, r1 = 0, r2 = 0;
  __device__ ProbeSeq4(uint64_t h1, uint64_t h2, const FastMod63& f) {
    v1 = h1 & 0x7FFFFFFFFFFFFFFFULL;
    v2 = h2 & 0x7FFFFFFFFFFFFFFFULL;
    r1 = fastmod63(v1, f);
    r2 = fastmod63(v2, f);
    v = v1;
    idx = r1;
  }
  __device__ void next(int t, const FastMod63& f) {
    const uint64_t b = (t & 1) ? v1 : v2, rb = (t & 1) ? r1 : r2;
    const uint64_t s = v + b;
    uint64_t x = idx + rb;
    x = x >= f.d ? x - f.d : x;
    if (s >> 63) x = x >= f.r63 ? x - f.r63 : x + (f.d - f.r63);
    v = s & 0x7FFFFFFFFFFFFFFFULL;
    idx = x;
  }
};

// k = 7 as a constant, as in the insert's sa1 instance for C3 (KC = 7): the step loop unrolled
template <int MODE>
__global__ __launch_bounds__(256) void chain_kernel(uint64_t keys_per_lane, FastMod63 fm, int, uint64_t* out) {
  constexpr int k = 7;
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc = 0;
  for (uint64_t q = 0; q < keys_per_lane; ++q) {
    const uint64_t i = lane * keys_per_lane + q;
    const uint64_t w0 = i ^ 0x5EED0003ULL, w1 = rotl(i, 17) ^ 0xA5A5A5A5DEADBEEFULL;
    if (MODE == 0) {
      acc += w0 ^ w1;
      continue;
    }
    const uint64_t h1 = xxh64_16(w0, w1), h2 = farm_16(w0, w1);
    if (MODE == 1) {
      acc += h1 ^ h2;
      continue;
    }
    if (MODE == 2) {
      ProbeSeq4 ps(h1, h2, fm);
      for (int t = 0; t < k; ++t) {
        acc += ps.idx;
        if (t + 1 < k) ps.next(t, fm);
      }
      continue;
    }
    ProbeSeq ps;
    if (MODE == 4) {
      ps.v1 = h1 & 0x7FFFFFFFFFFFFFFFULL;
      ps.v2 = h2 & 0x7FFFFFFFFFFFFFFFULL;
      ps.init(fastmod63_big(ps.v1, fm), fastmod63_big(ps.v2, fm), fm);
    } else {
      ps = ProbeSeq(h1, h2, fm);
    }
    for (int t = 0; t < k; ++t) {
      acc += ps.idx;
      if (t + 1 < k) ps.next(t, fm);
    }
  }
  out[lane] = acc;
}

// Both mods on the same dividends: sampled key chains plus boundary values.
__global__ __launch_bounds__(256) void check_kernel(uint64_t keys_per_lane, FastMod63 fm, int k,
                                                     unsigned long long* bad) {
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t nbad = 0;
  for (uint64_t q = 0; q < keys_per_lane; ++q) {
    const uint64_t i = lane * keys_per_lane + q;
    const uint64_t w0 = i ^ 0x5EED0003ULL, w1 = rotl(i, 17) ^ 0xA5A5A5A5DEADBEEFULL;
    const uint64_t h1 = xxh64_16(w0, w1), h2 = farm_16(w0, w1);
    ProbeSeq4 a(h1, h2, fm);
    ProbeSeq b(h1, h2, fm);
    for (int t = 0; t < k; ++t) {
      nbad += a.idx != b.idx;
      if (t + 1 < k) {
        a.next(t, fm);
        b.next(t, fm);
      }
    }
    // boundary dividends: m d + {-2..2} for m spread over [0, 2^63 / d]
    const uint64_t mmax = 0x7FFFFFFFFFFFFFFFULL / fm.d;
    const uint64_t m = (i * 0x9E3779B97F4A7C15ULL) % (mmax + 1);
    for (int e = -2; e <= 2; ++e) {
      const uint64_t x = m * fm.d + (uint64_t)(int64_t)e;
      if (x > 0x7FFFFFFFFFFFFFFFULL) continue;
      nbad += fastmod63(x, fm) != fastmod63_big(x, fm);
    }
    const uint64_t top = 0x7FFFFFFFFFFFFFFFULL - (i & 0xFFFF);
    nbad += fastmod63(top, fm) != fastmod63_big(top, fm);
  }
  if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

template <int MODE>
static double run(uint64_t kpl, int blocks, const FastMod63& fm, int k, uint64_t* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(chain_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, kpl, fm, k, out);
  float t[3];
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(chain_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, kpl, fm, k, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t[r], a, b));
  }
  float lo = t[0] < t[1] ? t[0] : t[1], hi = t[0] < t[1] ? t[1] : t[0];
  return t[2] < lo ? lo : (t[2] > hi ? hi : t[2]);
}

int main(int argc, char** argv) {
  const uint64_t size = argc > 1 ? strtoull(argv[1], 0, 10) : 9585058378ULL;
  const int k = 7;  // the timed kernels' constant
  const FastMod63 fm = host_fastmod(size);
  const int blocks = 256 * 16;  // 4 workgroups (16 waves) per CU
  const double lanes = (double)blocks * 256;
  const uint64_t kpl = (uint64_t)(1e9 / lanes) + 1;
  uint64_t* out;
  CK(hipMalloc(&out, (size_t)lanes * 8));
  unsigned long long* bad;
  CK(hipMalloc(&bad, 8));
  CK(hipMemset(bad, 0, 8));
  const double scale = 1e9 / (kpl * lanes);
  printf("{\"size\": %llu, \"k\": %d, \"keys\": 1e9", (unsigned long long)size, k);
  printf(", \"keywords_ms\": %.3f", run<0>(kpl, blocks, fm, k, out) * scale);
  printf(", \"hashes_ms\": %.3f", run<1>(kpl, blocks, fm, k, out) * scale);
  printf(", \"probes_round4_ms\": %.3f", run<2>(kpl, blocks, fm, k, out) * scale);
  printf(", \"probes_ms\": %.3f", run<3>(kpl, blocks, fm, k, out) * scale);
  printf(", \"probes_big_mods_ms\": %.3f", run<4>(kpl, blocks, fm, k, out) * scale);
  hipLaunchKernelGGL(check_kernel, dim3(blocks), dim3(256), 0, 0, (uint64_t)16, fm, k, bad);
  unsigned long long nb = 0;
  CK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
  printf(", \"mismatches\": %llu, \"checked_keys\": %.0f}\n", nb, lanes * 16);
  return nb ? 1 : 0;
}
