// rsk_hllcount.h -- the PFCOUNT arithmetic shared by the count kernels
// (rsk_hll.hip) and the grouped add's fused estimate (rsk_bloom_part.hip):
// Redis 3.2.0 hllCount (hyperloglog.c) in FP64, compiled -ffp-contract=off.
#pragma once

#include "rsk_device.h"

namespace rsk {

RSK_DEV double pe(uint32_t r) {  // 2^-r, exact
  return __longlong_as_double((long long)((uint64_t)(1023 - r) << 52));
}

// hllCount tail (Redis 3.2.0), FP64, compiled with -ffp-contract=off.
// lc[ez] = m*log(m/ez) from the host libm.
RSK_DEV uint64_t hll_estimate(double E, int ez, const double* __restrict__ lc) {
  const double m = HLL_REGS;
  double alpha = 0.7213 / (1 + 1.079 / m);
  E = (1 / E) * alpha * m * m;
  if (E < m * 2.5 && ez != 0) {
    E = lc[ez];
  } else if (E < 72000) {
    double bias = 5.9119 * 1.0e-18 * (E * E * E * E) - 1.4253 * 1.0e-12 * (E * E * E) +
                  1.2940 * 1.0e-7 * (E * E) - 5.2921 * 1.0e-3 * E + 83.3216;
    E -= E * (bias / 100);
  }
  return (uint64_t)E;
}

// Redis sums 2^-reg in an encoding-specific order.  All orders agree when
// every partial sum is exact: the terms are multiples of 2^-rmax, so every
// partial sum below 2^(53-rmax) is an exact double.  The kernels therefore
// sum in any order in FP64, each term built directly as the bits of 2^-r,
// and compare the total with that bound.  Rounding is monotone and the
// bound is representable, so the computed total reaches it iff the exact
// total does; only then is Redis's order replayed serially (dense: groups
// of 16; raw: u64 words).  Sparse keys always pass (registers <= 32).
struct SumD {
  double t;       // sum over all registers of 2^-r (a zero register adds 1)
  uint32_t ez;    // zero registers
  uint32_t rmax;  // largest register
};

RSK_DEV void acc_word(SumD& s, uint32_t w) {
  // bit 7 of a byte of z is set exactly where that byte of w is zero
  const uint32_t z = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu);
  s.ez += __popc(z);
  const uint32_t r0 = w & 0xFFu, r1 = (w >> 8) & 0xFFu, r2 = (w >> 16) & 0xFFu, r3 = w >> 24;
  const uint32_t m01 = r0 > r1 ? r0 : r1, m23 = r2 > r3 ? r2 : r3;
  const uint32_t m = m01 > m23 ? m01 : m23;
  s.rmax = m > s.rmax ? m : s.rmax;
  s.t += (pe(r0) + pe(r1)) + (pe(r2) + pe(r3));
}

// Registers below 15 (sparse sketches: the grouped add's fresh rows): 2^-r
// as the integer 2^(14-r), two bytes per packed 16-bit shift summed by a
// dot product -- 15 VALU per word against acc_word's ~25.  `big` flags a
// byte of 15 or more (the caller then sums with acc_word).  A lane's 256
// bytes sum below 2^22, a sketch's below 2^28; t = s 2^-14 is exact and,
// with every register below 15, below 2^(53-14).
struct SumQ {
  uint32_t s;    // sum of 2^(14-r)
  uint32_t ez;   // zero registers
  uint32_t big;  // bit 7 of a byte set: a register >= 15
};
RSK_DEV void accq_word(SumQ& q, uint32_t w) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  const us2 base = {0x4000, 0x4000}, one = {1, 1};
  const us2 r01 = __builtin_bit_cast(us2, __builtin_amdgcn_perm(0u, w, 0x0c010c00u));  // bytes 0, 1 -> halves
  const us2 r23 = __builtin_bit_cast(us2, __builtin_amdgcn_perm(0u, w, 0x0c030c02u));  // bytes 2, 3 -> halves
  q.s = __builtin_amdgcn_udot2(base >> r01, one, q.s, false);
  q.s = __builtin_amdgcn_udot2(base >> r23, one, q.s, false);
  const uint32_t z = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu);
  q.ez += __popc(z);
  q.big |= (w + 0x71717171u) & 0x80808080u;  // bytes <= 63: no carry between bytes
}

RSK_DEV SumD wave_reduce(SumD s) {
  for (int off = 32; off > 0; off >>= 1) {
    s.t += __shfl_down(s.t, off, 64);
    s.ez += __shfl_down(s.ez, off, 64);
    const uint32_t o = __shfl_down(s.rmax, off, 64);
    s.rmax = o > s.rmax ? o : s.rmax;
  }
  return s;
}

// Every summation order gives s.t exactly (see above).
RSK_DEV bool exact_total(const SumD& s) {
  return s.t < __longlong_as_double((long long)((uint64_t)(1023 + 53 - s.rmax) << 52));  // 2^(53-rmax)
}

}  // namespace rsk
