// rsk_hll_io.hip -- the Redis wire format of many HLL keys per call: batched
// GET / SET of the "HYLL" strings (rsk_hll_export_redis_batch /
// rsk_hll_import_redis_batch), the checkpoint of a grouped pool (SURVEY 5,
// 8f-1).  One wave per key, its 16384 registers staged in LDS:
//   export : (encoded once into a fixed slot per key, then packed to its
//            offset) the row's run starts compacted in order (four registers
//            per lane per step, slots from ballots), then either the canonical
//            sparse opcodes (Redis hyperloglog.c: ZERO 00xxxxxx run 1..64,
//            XZERO 01xxxxxx yyyyyyyy run 1..16384, VAL 1vvvvvxx value 1..32
//            run 1..4; maximal runs cut into the longest opcodes, as
//            encode_sparse in rsk_api.hip) one run per lane, or the 6-bit
//            LSB-first dense packing (HLL_DENSE_SET_REGISTER), four registers
//            per lane at a time;
//   import : the sparse opcode stream parsed 64 bytes per step (which bytes
//            are XZERO second bytes follows from the last non-XZERO byte
//            before each lane; run lengths prefix-summed across the wave),
//            checked like rsk_hll_import_redis (every register covered
//            exactly once), then written into the pool row.
#include "rsk_internal.h"

#include <utility>

namespace rsk {

constexpr uint32_t IO_DENSE = 12304;        // HLL_DENSE_SIZE: 16-byte header + 12288
constexpr uint32_t IO_SPARSE_MAX = 3000;    // server.hll_sparse_max_bytes (whole string)

// This wave's LDS writes are visible to its other lanes (one wave: in order).
RSK_DEV void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Lane l gets lane l - 1's x, lane 0 gets lane0 (DPP wave_shr:1, no LDS trip).
RSK_DEV uint32_t wave_shr1(uint32_t x, uint32_t lane0) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)x, 0x138, 0xF, 0xF, false);
}
// Set bits of b in lanes below this one, plus acc.
RSK_DEV uint32_t lanes_below(uint64_t b, uint32_t acc) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, acc));
}

// The export's wave: the row and its run starts in order.  Every run is at
// least one payload byte, so a row of more runs than IO_RUNS is dense.
constexpr uint32_t IO_RUNS = IO_SPARSE_MAX - 16;
struct ExWave {
  uint8_t row[HLL_REGS];
  uint16_t start[IO_RUNS];
};

// Pass 1: the run starts of the row, compacted in order into S.start (a
// register starts a run when it differs from the one before; register 0
// always does).  Four registers per lane per step (one dword of the row, the
// next step's read issued ahead): lane l of step t holds registers 256 t + 4 l
// .. + 3; a start's slot is the starts in the step's four ballots below this
// lane (mbcnt) plus the lane's own earlier ones.  Returns the number of runs
// (stops counting past IO_RUNS: dense); *big: a register exceeds 32 (VAL
// holds 1..32: no sparse form), valid when the count is at most IO_RUNS.
RSK_DEV uint32_t row_starts(ExWave& S, uint32_t lane, bool* big) {
  const uint32_t* r32 = reinterpret_cast<const uint32_t*>(S.row);
  uint32_t carry = 0x100u, o = 0, wn = r32[lane];
  bool b = false;
  for (uint32_t t = 0; t < HLL_REGS / 256; ++t) {
    const uint32_t w = wn;
    wn = r32[64 * ((t + 1) & 63) + lane];
    const uint32_t r0 = w & 0xFFu, r1 = (w >> 8) & 0xFFu, r2 = (w >> 16) & 0xFFu, r3 = w >> 24;
    const uint32_t prev = wave_shr1(r3, carry);
    carry = (uint32_t)__builtin_amdgcn_readlane((int)r3, 63);
    b |= ((w + 0x5F5F5F5Fu) & 0x80808080u) != 0;  // a byte of 33 .. 63 (registers are at most 63)
    const bool n[4] = {r0 != prev, r1 != r0, r2 != r1, r3 != r2};
    const uint64_t b0 = __ballot(n[0]), b1 = __ballot(n[1]), b2 = __ballot(n[2]), b3 = __ballot(n[3]);
    uint32_t at = lanes_below(b3, lanes_below(b2, lanes_below(b1, lanes_below(b0, o))));
    const uint32_t j0 = 256 * t + 4 * lane;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (n[i] && at < IO_RUNS) S.start[at] = (uint16_t)(j0 + i);
      at += n[i] ? 1u : 0u;
    }
    o += (uint32_t)(__popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3));
    if (o > IO_RUNS) break;  // (uniform)
  }
  *big = __ballot(b) != 0;
  return o;
}

// Pass 2: the canonical sparse payload (Redis hyperloglog.c), one run per
// lane, 64 runs per step: a zero run of L registers is ZERO (L - 1) when L <=
// 64, else XZERO's two bytes; a run of value v is ceil(L / 4) VAL opcodes of
// 4 registers, the last one of the remainder.  Each run's bytes land at the
// exclusive scan of the bytes per run.  Returns the payload length, or a
// count past IO_RUNS (stopped early) when it does not fit a sparse string.
RSK_DEV uint32_t runs_encode(const ExWave& S, uint32_t lane, uint32_t R, uint8_t* __restrict__ dst) {
  uint32_t o = 0;
  for (uint32_t rb = 0; rb < R; rb += 64) {
    const uint32_t r = rb + lane;
    const bool in = r < R;
    const uint32_t s = in ? S.start[r] : 0u, e = r + 1 < R ? S.start[r + 1] : (uint32_t)HLL_REGS;
    const uint32_t v = S.row[s], L = e - s;
    const uint32_t nb = !in ? 0u : v ? (L + 3) >> 2 : (L > 64 ? 2u : 1u);
    uint32_t x = nb;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    const uint32_t tot = (uint32_t)__shfl((int)x, 63, 64);
    if (o + tot > IO_RUNS) return o + tot;  // (uniform)
    const uint32_t at = o + x - nb;
    const uint32_t zb0 = L <= 64 ? L - 1 : 0x40u | ((L - 1) >> 8);
    for (uint32_t q = 0; __ballot(q < nb) != 0; ++q)
      if (q < nb) {
        const uint32_t rl = min(L - 4 * q, 4u);
        dst[at + q] = (uint8_t)(v ? 0x80u | ((v - 1) << 2) | (rl - 1) : q == 0 ? zb0 : ((L - 1) & 0xFFu));
      }
    o += tot;
  }
  return o;
}

// Export (rsk_hll_export_redis_batch): key i encoded once, into its slot
// slots + i IO_DENSE (16-byte aligned), its length in len[i] (| 1 << 31 for a
// key that stays sparse: want_sparse and it fits -- registers <= 32, string
// <= 3000 bytes -- else the dense 12304 bytes).  The sparse payload is written
// while it is counted; a payload that turns out too long is overwritten by the
// dense form.  hll_export_pack then moves the strings to their offsets.
// A row in registers, 16 bytes x 16 per lane (a native vector type and
// constant indices from the start: the array stays in VGPRs across the key
// loop, where uint4's struct copies kept it in scratch).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <size_t... U>
RSK_DEV void row_regs_load(u32x4 (&nx)[sizeof...(U)], const uint8_t* __restrict__ src, uint32_t lane,
                           std::index_sequence<U...>) {
  const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
  ((nx[U] = s4[lane + 64 * U]), ...);
}
template <size_t... U>
RSK_DEV void row_regs_store(const u32x4 (&nx)[sizeof...(U)], ExWave& S, uint32_t lane, std::index_sequence<U...>) {
  u32x4* d4 = reinterpret_cast<u32x4*>(S.row);
  ((d4[lane + 64 * U] = nx[U]), ...);
}

__global__ __launch_bounds__(64) void hll_export_kernel(const uint8_t* __restrict__ regs,
                                                        const uint64_t* __restrict__ card,
                                                        const uint64_t* __restrict__ ids,
                                                        const uint8_t* __restrict__ want_sparse, uint32_t n,
                                                        uint32_t* __restrict__ len, uint8_t* __restrict__ slots) {
  __shared__ ExWave S;  // one wave per workgroup: LDS is what bounds the waves per CU
  const uint32_t lane = threadIdx.x;
  constexpr int NV = HLL_REGS / 16 / 64;
  u32x4 nx[NV];  // the next key's row, loaded while this key is encoded
  const auto U = std::make_index_sequence<NV>{};
  uint32_t i = blockIdx.x;
  row_regs_load(nx, regs + ids[i < n ? i : 0] * HLL_REGS, lane, U);
  for (; i < n; i += gridDim.x) {  // wave-uniform
    const uint64_t id = ids[i];
    uint8_t* d = slots + (uint64_t)i * IO_DENSE;
    row_regs_store(nx, S, lane, U);
    wave_lds_sync();
    row_regs_load(nx, regs + ids[i + gridDim.x < n ? i + gridDim.x : i] * HLL_REGS, lane, U);
    bool sparse = want_sparse[i] != 0;
    uint32_t pl = 0;
    if (sparse) {
      bool big;
      const uint32_t R = row_starts(S, lane, &big);
      sparse = !big && R <= IO_RUNS;
      if (sparse) {
        wave_lds_sync();
        pl = runs_encode(S, lane, R, d + 16);  // (a longer one is dense: the slot stays in bounds)
        sparse = pl <= IO_RUNS;
      }
    }
    if (lane < 16) {
      const uint64_t cv = card[id];
      const uint8_t hdr = lane < 4 ? (uint8_t)"HYLL"[lane] : lane == 4 ? (uint8_t)(sparse ? 1 : 0)
                          : lane < 8 ? (uint8_t)0 : (uint8_t)(cv >> (8 * (lane - 8)));
      d[lane] = hdr;
    }
    if (!sparse) {
      // the register stream, 6 bits each, LSB first: registers 4g .. 4g + 3 are payload bytes 3g .. 3g + 2
      const uint32_t* r32 = reinterpret_cast<const uint32_t*>(S.row);
      for (uint32_t g = lane; g < HLL_REGS / 4; g += 64) {
        const uint32_t w = r32[g];
        const uint32_t bits = (w & 63u) | ((w >> 8) & 63u) << 6 | ((w >> 16) & 63u) << 12 | ((w >> 24) & 63u) << 18;
        uint8_t* q = d + 16 + 3 * g;
        q[0] = (uint8_t)bits;
        q[1] = (uint8_t)(bits >> 8);
        q[2] = (uint8_t)(bits >> 16);
      }
    }
    if (lane == 0) len[i] = sparse ? (0x80000000u | (16 + pl)) : IO_DENSE;
    wave_lds_sync();  // the row is read by every lane before the next key's load
  }
}

// String i (slot i, len[i] bytes) to out + pos[i]: one workgroup per string
// at a time, bytes in order across the lanes (the stores of a wave fill lines).
__global__ __launch_bounds__(256) void hll_export_pack_kernel(const uint8_t* __restrict__ slots,
                                                              const uint32_t* __restrict__ len,
                                                              const uint64_t* __restrict__ pos, uint32_t n,
                                                              uint8_t* __restrict__ out) {
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t L = len[i] & 0x7FFFFFFFu;
    const uint8_t* src = slots + (uint64_t)i * IO_DENSE;
    uint8_t* dst = out + pos[i];
    for (uint32_t b = threadIdx.x; b < L; b += 256) dst[b] = src[b];
  }
}

// One opcode from its first byte (and the next, for XZERO): run length; *val
// its register value (0 for ZERO / XZERO); *two: it takes two bytes.
RSK_DEV uint32_t sp_op(uint32_t b, uint32_t b1, uint32_t* val, bool* two) {
  *two = (b & 0xC0u) == 0x40u;
  if ((b & 0xC0u) == 0) {
    *val = 0;
    return (b & 0x3Fu) + 1;
  }
  if (*two) {
    *val = 0;
    return (((b & 0x3Fu) << 8) | b1) + 1;
  }
  *val = ((b >> 2) & 0x1Fu) + 1;
  return (b & 3u) + 1;
}

// Inclusive sum over the wave on the DPP path: within each 16-lane row
// (row_shr 1, 2, 4, 8, zeros shifted in), then row 0's total into row 1 and
// row 2's into row 3 (row_bcast:15), rows 0-1's into rows 2-3 (row_bcast:31).
RSK_DEV uint32_t wave_incl_add(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  return x;
}

// Import (rsk_hll_import_redis_batch): string i = data[off[i] .. off[i+1]),
// its 16-byte header already checked on the host.  APPLY false: the check
// pass over sparse strings -- every register covered exactly once (else
// atomicMin(err, i)), canon[i] = the payload is what the export would write
// (no two zero opcodes in a row, no XZERO of 64 or fewer, a VAL shorter than
// 4 never followed by a VAL of its value).  APPLY (and no error): every
// string with apply[i] set is decoded into row ids[i] and its card bytes.
// A sparse payload of at most IO_SB bytes is first copied into LDS with
// 16-byte loads all in flight together, then parsed from there (parsing
// from global memory waited a full load latency per 64-byte step); a longer
// one is parsed from global memory.  One wave per workgroup.
constexpr uint32_t IO_SB = 4096;
template <bool APPLY>
struct ImWave;
template <>
struct ImWave<false> {
  uint8_t sb[IO_SB + 32];
};
template <>
struct ImWave<true> {
  uint8_t row[HLL_REGS];
  uint8_t sb[IO_SB + 32];
};
template <bool APPLY>
__global__ __launch_bounds__(64) void hll_import_kernel(const uint8_t* __restrict__ data,
                                                        const uint64_t* __restrict__ off,
                                                        const uint64_t* __restrict__ ids,
                                                        const uint8_t* __restrict__ apply, uint32_t n,
                                                        uint8_t* __restrict__ regs, uint64_t* __restrict__ card,
                                                        uint8_t* __restrict__ canon,
                                                        unsigned long long* __restrict__ err, uint32_t i0) {
  __shared__ __attribute__((aligned(16))) ImWave<APPLY> S;
  const uint32_t lane = threadIdx.x;
  if (APPLY && *err != ~0ull) return;  // a string failed the check: nothing is written
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {  // wave-uniform
    if (APPLY && !apply[i]) continue;
    const uint8_t* s = data + off[i];
    const uint32_t slen = (uint32_t)(off[i + 1] - off[i]);
    const bool dense = s[4] == 0;
    if (!APPLY && dense) continue;  // nothing to check (exact length checked on the host)
    const uint8_t* p = s + 16;
    const uint32_t plen = slen - 16;
    if constexpr (APPLY) {
      if (dense) {
        uint8_t* row = regs + ids[i] * HLL_REGS;
        // registers 16q .. 16q + 15 = payload bytes 12q .. 12q + 11
#pragma unroll 4
        for (uint32_t q = lane; q < HLL_REGS / 16; q += 64) {
          const uint8_t* b = p + 12 * q;
          const uint64_t lo = (uint64_t)ld_u32(b) | (uint64_t)ld_u32(b + 4) << 32;
          const uint32_t hi = ld_u32(b + 8);
          uint32_t w[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            uint32_t x = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const uint32_t bit = 6 * (4 * r + t);
              const uint32_t v = bit + 6 <= 64 ? (uint32_t)(lo >> bit) & 63u
                                 : bit >= 64 ? (hi >> (bit - 64)) & 63u
                                             : (uint32_t)((lo >> bit) | ((uint64_t)hi << (64 - bit))) & 63u;
              x |= v << (8 * t);
            }
            w[r] = x;
          }
          reinterpret_cast<uint4*>(row)[q] = make_uint4(w[0], w[1], w[2], w[3]);
        }
        if (lane == 0) card[ids[i]] = ld_u64(s + 8);
        continue;
      }
      uint4* d4 = reinterpret_cast<uint4*>(S.row);
      for (uint32_t u = lane; u < HLL_REGS / 16; u += 64) d4[u] = make_uint4(0, 0, 0, 0);
    }
    // the payload into LDS (16-byte aligned loads around it: d_data has slack past the end)
    const bool staged = plen <= IO_SB;
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u);
    if (staged) {
      const uint4* g4 = reinterpret_cast<const uint4*>(p - sh);
      const uint32_t n4 = (sh + plen + 15) / 16;
      uint4 v[IO_SB / 16 / 64 + 1];
#pragma unroll
      for (uint32_t u = 0; u < IO_SB / 16 / 64 + 1; ++u) {
        const uint32_t c = lane + 64 * u;
        v[u] = c < n4 ? g4[c] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (uint32_t u = 0; u < IO_SB / 16 / 64 + 1; ++u) {
        const uint32_t c = lane + 64 * u;
        if (c < n4 && 16 * c < IO_SB + 32) reinterpret_cast<uint4*>(S.sb)[c] = v[u];
      }
    }
    wave_lds_sync();
    auto byte_at = [&](uint32_t q) -> uint32_t { return staged ? S.sb[sh + q] : p[q]; };
    uint32_t at = 0, cin = 0;  // registers covered so far; byte 0 of the step is an XZERO second byte
    bool ok = true, can = true;
    for (uint32_t c0 = 0; c0 < plen; c0 += 64) {
      const uint32_t q = c0 + lane;
      const bool in = q < plen;
      const uint32_t b = in ? byte_at(q) : 0u;
      const bool isx = in && (b & 0xC0u) == 0x40u;
      // byte l is a second byte iff an odd number of XZERO first bytes precede it back to the
      // last byte that cannot start one (or to the step's start, whose state is cin)
      const uint64_t z = __ballot(!isx), zb = z & ((1ull << lane) - 1);
      const uint32_t cont = zb ? ((lane - (63 - (uint32_t)__clzll(zb)) - 1) & 1u) : ((cin ^ lane) & 1u);
      cin = z ? ((64 - (63 - (uint32_t)__clzll(z)) - 1) & 1u) : cin;
      const bool st = in && !cont;
      uint32_t val = 0, run = 0;
      bool two = false;
      if (st) {
        const uint32_t b1 = q + 1 < plen ? byte_at(q + 1) : 0u;
        run = sp_op(b, b1, &val, &two);
        if (two && q + 1 >= plen) ok = false;  // XZERO cut by the end of the string
        if constexpr (!APPLY) {
          // canonical form: the export's encoder would emit exactly this opcode here
          if (two && run <= 64) can = false;
          const uint32_t qn = q + (two ? 2 : 1);
          if (qn < plen) {
            uint32_t nv = 0;
            bool ntwo = false;
            (void)sp_op(byte_at(qn), qn + 1 < plen ? byte_at(qn + 1) : 0u, &nv, &ntwo);
            if (val == 0 && nv == 0) can = false;                  // two zero runs in a row
            if (val != 0 && nv == val && run < 4) can = false;     // a VAL run cut short
          }
        }
      }
      // register position of each opcode: exclusive prefix of the run lengths
      const uint32_t x = wave_incl_add(run);
      const uint32_t first = at + x - run;
      if constexpr (APPLY)
        if (st && val != 0 && first + run <= (uint32_t)HLL_REGS)
          for (uint32_t r = 0; r < run; ++r) S.row[first + r] = (uint8_t)val;
      at += (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
      if (at > (uint32_t)HLL_REGS) at = HLL_REGS + 1;  // (no wrap on adversarial input)
    }
    ok = __ballot(!ok) == 0 && at == (uint32_t)HLL_REGS;
    can = __ballot(!can) == 0;
    if constexpr (!APPLY) {
      if (lane == 0) {
        canon[i] = can ? 1 : 0;
        if (!ok) atomicMin(err, (unsigned long long)(i0 + i));  // (i0: the chunk's first string in the call)
      }
    } else {
      wave_lds_sync();
      uint8_t* row = regs + ids[i] * HLL_REGS;
      const uint4* s4 = reinterpret_cast<const uint4*>(S.row);
      for (uint32_t u = lane; u < HLL_REGS / 16; u += 64) reinterpret_cast<uint4*>(row)[u] = s4[u];
      if (lane == 0) card[ids[i]] = ld_u64(s + 8);
    }
    wave_lds_sync();  // this string's LDS reads are done before the next string's writes
  }
}

void hll_export_launch(rsk_ctx* c, const uint8_t* d_regs, const uint64_t* d_card, const uint64_t* d_ids,
                       const uint8_t* d_want_sparse, uint32_t n, uint32_t* d_len, uint8_t* d_slots) {
  if (!n) return;
  ProfScope ps(c, "hll_export_encode");
  const uint32_t blocks = std::min<uint32_t>(n, (uint32_t)c->num_cus * 7);  // 22 KB LDS per wave: 7 waves per CU
  hipLaunchKernelGGL(hll_export_kernel, dim3(blocks), dim3(64), 0, c->stream, d_regs, d_card, d_ids, d_want_sparse,
                     n, d_len, d_slots);
  RSK_CHECK_LAUNCH("hll_export");
}

void hll_export_pack_launch(rsk_ctx* c, const uint8_t* d_slots, const uint32_t* d_len, const uint64_t* d_pos,
                            uint32_t n, uint8_t* d_out) {
  if (!n) return;
  ProfScope ps(c, "hll_export_pack");
  const uint32_t blocks = std::min<uint32_t>(n, (uint32_t)c->num_cus * 8);
  hipLaunchKernelGGL(hll_export_pack_kernel, dim3(blocks), dim3(256), 0, c->stream, d_slots, d_len, d_pos, n, d_out);
  RSK_CHECK_LAUNCH("hll_export_pack");
}

// The import's decode per chunk (overlapped with the next chunk's upload) stays
// all-or-nothing: before a chunk is decoded, the rows (and card words) its
// strings will replace are copied aside (bak row i for string i), and if any
// string of the call fails its check they are copied back.  One workgroup per
// string with apply[i] set, 16-byte lanes.
template <bool RESTORE>
__global__ __launch_bounds__(256) void hll_rows_bak_kernel(uint4* __restrict__ regs, uint64_t* __restrict__ card,
                                                           const uint64_t* __restrict__ ids,
                                                           const uint8_t* __restrict__ apply, uint32_t n,
                                                           uint4* __restrict__ bak, uint64_t* __restrict__ bak_card,
                                                           const unsigned long long* __restrict__ err) {
  constexpr uint32_t ROW_U4 = HLL_REGS / 16;
  if (RESTORE && *err == ~0ull) return;  // every string passed: nothing to undo
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    if (!apply[i]) continue;
    uint4* row = regs + ids[i] * ROW_U4;
    uint4* b = bak + (uint64_t)i * ROW_U4;
    for (uint32_t q = threadIdx.x; q < ROW_U4; q += 256) {
      if (RESTORE) row[q] = b[q];
      else b[q] = row[q];
    }
    if (threadIdx.x == 0) {
      if (RESTORE) card[ids[i]] = bak_card[i];
      else bak_card[i] = card[ids[i]];
    }
  }
}

void hll_rows_bak_launch(rsk_ctx* c, bool restore, uint8_t* d_regs, uint64_t* d_card, const uint64_t* d_ids,
                         const uint8_t* d_apply, uint32_t n, uint8_t* d_bak, uint64_t* d_bak_card,
                         const unsigned long long* d_err) {
  if (!n) return;
  ProfScope ps(c, restore ? "hll_import_restore" : "hll_import_backup");
  const dim3 g(std::min<uint32_t>(n, (uint32_t)c->num_cus * 8)), b(256);
  if (restore)
    hipLaunchKernelGGL(hll_rows_bak_kernel<true>, g, b, 0, c->stream, reinterpret_cast<uint4*>(d_regs), d_card, d_ids,
                       d_apply, n, reinterpret_cast<uint4*>(d_bak), d_bak_card, d_err);
  else
    hipLaunchKernelGGL(hll_rows_bak_kernel<false>, g, b, 0, c->stream, reinterpret_cast<uint4*>(d_regs), d_card, d_ids,
                       d_apply, n, reinterpret_cast<uint4*>(d_bak), d_bak_card, d_err);
  RSK_CHECK_LAUNCH("hll_rows_bak");
}

void hll_import_launch(rsk_ctx* c, const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_ids,
                       const uint8_t* d_apply, uint32_t n, uint8_t* d_regs, uint64_t* d_card, uint8_t* d_canon,
                       unsigned long long* d_err, uint32_t i0) {
  if (!n) return;
  ProfScope ps(c, d_apply ? "hll_import_write" : "hll_import_check");
  // one wave per workgroup: the check pass holds 4 KiB of LDS (24 waves per CU), the decode 20 KiB (7 per CU)
  if (d_apply)
    hipLaunchKernelGGL(hll_import_kernel<true>, dim3(std::min<uint32_t>(n, (uint32_t)c->num_cus * 7)), dim3(64), 0,
                       c->stream, d_data, d_off, d_ids, d_apply, n, d_regs, d_card, d_canon, d_err, i0);
  else
    hipLaunchKernelGGL(hll_import_kernel<false>, dim3(std::min<uint32_t>(n, (uint32_t)c->num_cus * 24)), dim3(64), 0,
                       c->stream, d_data, d_off, d_ids, d_apply, n, d_regs, d_card, d_canon, d_err, i0);
  RSK_CHECK_LAUNCH("hll_import");
}

}  // namespace rsk
