// rsk_hll_io.hip -- the Redis wire format of many HLL keys per call: batched
// GET / SET of the "HYLL" strings (rsk_hll_export_redis_batch /
// rsk_hll_import_redis_batch), the checkpoint of a grouped pool (SURVEY 5,
// 8f-1).  One wave per key, its 16384 registers staged in LDS:
//   export : (encoded once into a fixed slot per key, then packed to its
//            offset) the key's run structure (a start mask per 64 registers, the last
//            / first run start around each chunk), then either the canonical
//            sparse opcodes (Redis hyperloglog.c: ZERO 00xxxxxx run 1..64,
//            XZERO 01xxxxxx yyyyyyyy run 1..16384, VAL 1vvvvvxx value 1..32
//            run 1..4; maximal runs cut into the longest opcodes, as
//            encode_sparse in rsk_api.hip) or the 6-bit LSB-first dense
//            packing (HLL_DENSE_SET_REGISTER), one byte per lane at a time;
//   import : the sparse opcode stream parsed 64 bytes per step (which bytes
//            are XZERO second bytes follows from the last non-XZERO byte
//            before each lane; run lengths prefix-summed across the wave),
//            checked like rsk_hll_import_redis (every register covered
//            exactly once), then written into the pool row.
#include "rsk_internal.h"

namespace rsk {

constexpr uint32_t IO_T = 256;              // 4 waves: one key each
constexpr uint32_t IO_W = IO_T / 64;
constexpr uint32_t IO_NCH = HLL_REGS / 64;  // 64-register chunks of a row
constexpr uint32_t IO_DENSE = 12304;        // HLL_DENSE_SIZE: 16-byte header + 12288
constexpr uint32_t IO_SPARSE_MAX = 3000;    // server.hll_sparse_max_bytes (whole string)

struct IoWave {
  uint8_t row[HLL_REGS];
  uint64_t mask[IO_NCH];             // run starts of chunk k (bit l: register 64k + l)
  uint16_t lastw[IO_NCH];            // last run start at or before the end of chunk k
  uint16_t firstw[IO_NCH + 1];       // first run start at or after the beginning of chunk k (HLL_REGS: none)
};

// This wave's LDS writes are visible to its other lanes (one wave: in order).
RSK_DEV void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

RSK_DEV void row_load(IoWave& S, const uint8_t* __restrict__ src, uint32_t lane) {
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4 v[HLL_REGS / 16 / 64];
#pragma unroll
  for (int u = 0; u < HLL_REGS / 16 / 64; ++u) v[u] = s4[lane + 64 * u];
  uint4* d4 = reinterpret_cast<uint4*>(S.row);
#pragma unroll
  for (int u = 0; u < HLL_REGS / 16 / 64; ++u) d4[lane + 64 * u] = v[u];
  wave_lds_sync();
}

// Run starts of the row and their neighbours per chunk; true if any register
// exceeds 32 (no sparse form: VAL holds 1..32).
RSK_DEV bool row_runs(IoWave& S, uint32_t lane) {
  bool big = false;
  for (uint32_t k = 0; k < IO_NCH; ++k) {
    const uint32_t j = 64 * k + lane;
    const uint32_t v = S.row[j], p = j ? S.row[j - 1] : 0x100u;  // register 0 starts a run
    big |= v > 32;
    const uint64_t m = __ballot(v != p);
    if (lane == 0) S.mask[k] = m;
  }
  wave_lds_sync();
  // lane l: chunks 4l .. 4l + 3; prefix max of the last starts, suffix min of the first
  uint32_t last[4], first[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t k = 4 * lane + i;
    const uint64_t m = S.mask[k];
    last[i] = m ? 64 * k + 63 - (uint32_t)__clzll(m) : 0u;  // chunk 0 has register 0: the max is defined
    first[i] = m ? 64 * k + (uint32_t)__ffsll((long long)m) - 1 : (uint32_t)HLL_REGS;
  }
#pragma unroll
  for (int i = 1; i < 4; ++i) last[i] = max(last[i], last[i - 1]);
#pragma unroll
  for (int i = 2; i >= 0; --i) first[i] = min(first[i], first[i + 1]);
  uint32_t lx = last[3], fx = first[0];  // inclusive scans over lanes: max upward, min downward
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a = __shfl_up(lx, o, 64), b = __shfl_down(fx, o, 64);
    if (lane >= (uint32_t)o) lx = max(lx, a);
    if (lane + o < 64) fx = min(fx, b);
  }
  const uint32_t lprev = __shfl_up(lx, 1, 64), fnext = __shfl_down(fx, 1, 64);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    S.lastw[4 * lane + i] = (uint16_t)max(last[i], lane ? lprev : 0u);
    S.firstw[4 * lane + i] = (uint16_t)min(first[i], lane < 63 ? fnext : (uint32_t)HLL_REGS);
  }
  if (lane == 0) S.firstw[IO_NCH] = (uint16_t)HLL_REGS;
  wave_lds_sync();
  return __ballot(big) != 0;
}

// The canonical sparse payload of the row (after row_runs).  Every register
// contributes at most one byte -- a VAL opcode at every 4th register of a
// non-zero run, ZERO or the first XZERO byte at a zero run's start, the
// second XZERO byte at the 65th register of a zero run longer than 64 -- so
// register j's byte lands at the number of contributions before it.  dst
// null: the payload length only; bytes at or past dcap are not written.
RSK_DEV uint32_t row_sparse(const IoWave& S, uint32_t lane, uint8_t* __restrict__ dst, uint32_t dcap = 0xFFFFFFFFu) {
  uint32_t o = 0;
  const uint64_t lt = (1ull << lane) - 1, le = lane == 63 ? ~0ull : (2ull << lane) - 1;
  for (uint32_t k = 0; k < IO_NCH; ++k) {
    const uint32_t j = 64 * k + lane;
    const uint32_t v = S.row[j];
    const uint64_t m = S.mask[k], below = m & le, above = m & ~le;
    const uint32_t s = below ? 64 * k + 63 - (uint32_t)__clzll(below) : S.lastw[k ? k - 1 : 0];
    const uint32_t e = above ? 64 * k + (uint32_t)__ffsll((long long)above) - 1 : S.firstw[k + 1];
    const uint32_t L = e - s, p = j - s;
    bool emit;
    uint32_t byte;
    if (v == 0) {
      emit = p == 0 || (p == 64 && L > 64);
      byte = p == 0 ? (L <= 64 ? L - 1 : 0x40u | ((L - 1) >> 8)) : ((L - 1) & 0xFFu);
    } else {
      emit = (p & 3u) == 0;
      const uint32_t r = L - p < 4 ? L - p : 4u;
      byte = 0x80u | ((v - 1) << 2) | (r - 1);
    }
    const uint64_t em = __ballot(emit);
    const uint32_t at = o + (uint32_t)__popcll(em & lt);
    if (dst && emit && at < dcap) dst[at] = (uint8_t)byte;
    o += (uint32_t)__popcll(em);
  }
  return o;
}

// Export (rsk_hll_export_redis_batch): key i encoded once, into its slot
// slots + i IO_DENSE (16-byte aligned), its length in len[i] (| 1 << 31 for a
// key that stays sparse: want_sparse and it fits -- registers <= 32, string
// <= 3000 bytes -- else the dense 12304 bytes).  The sparse payload is written
// while it is counted; a payload that turns out too long is overwritten by the
// dense form.  hll_export_pack then moves the strings to their offsets.
__global__ __launch_bounds__(IO_T) void hll_export_kernel(const uint8_t* __restrict__ regs,
                                                          const uint64_t* __restrict__ card,
                                                          const uint64_t* __restrict__ ids,
                                                          const uint8_t* __restrict__ want_sparse, uint32_t n,
                                                          uint32_t* __restrict__ len, uint8_t* __restrict__ slots) {
  __shared__ IoWave SW[IO_W];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  IoWave& S = SW[wv];
  for (uint32_t i = blockIdx.x * IO_W + wv; i < n; i += gridDim.x * IO_W) {  // wave-uniform
    const uint64_t id = ids[i];
    uint8_t* d = slots + (uint64_t)i * IO_DENSE;
    row_load(S, regs + id * HLL_REGS, lane);
    bool sparse = want_sparse[i] != 0;
    uint32_t pl = 0;
    if (sparse) {
      sparse = !row_runs(S, lane);
      if (sparse) {
        pl = row_sparse(S, lane, d + 16, IO_SPARSE_MAX - 16);  // (a longer one is dense: the slot stays in bounds)
        sparse = 16 + pl <= IO_SPARSE_MAX;
      }
    }
    if (lane < 16) {
      const uint64_t cv = card[id];
      const uint8_t hdr = lane < 4 ? (uint8_t)"HYLL"[lane] : lane == 4 ? (uint8_t)(sparse ? 1 : 0)
                          : lane < 8 ? (uint8_t)0 : (uint8_t)(cv >> (8 * (lane - 8)));
      d[lane] = hdr;
    }
    if (!sparse) {
      // payload byte b = bits 8b .. 8b + 7 of the register stream (6 bits each, LSB first)
      for (uint32_t b = lane; b < IO_DENSE - 16; b += 64) {
        const uint32_t bit = 8 * b, j = bit / 6, fb = bit % 6;
        const uint32_t w = (S.row[j] & 63u) | (j + 1 < (uint32_t)HLL_REGS ? (uint32_t)(S.row[j + 1] & 63u) << 6 : 0u);
        d[16 + b] = (uint8_t)(w >> fb);
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

// Import (rsk_hll_import_redis_batch): string i = data[off[i] .. off[i+1]),
// its 16-byte header already checked on the host.  apply null: the check
// pass over sparse strings -- every register covered exactly once (else
// atomicMin(err, i)), canon[i] = the payload is what the export would write
// (no two zero opcodes in a row, no XZERO of 64 or fewer, a VAL shorter than
// 4 never followed by a VAL of its value).  apply given (and no error): every
// string with apply[i] set is decoded into row ids[i] and its card bytes.
__global__ __launch_bounds__(IO_T) void hll_import_kernel(const uint8_t* __restrict__ data,
                                                          const uint64_t* __restrict__ off,
                                                          const uint64_t* __restrict__ ids,
                                                          const uint8_t* __restrict__ apply, uint32_t n,
                                                          uint8_t* __restrict__ regs, uint64_t* __restrict__ card,
                                                          uint8_t* __restrict__ canon,
                                                          unsigned long long* __restrict__ err) {
  __shared__ IoWave SW[IO_W];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  IoWave& S = SW[wv];
  if (apply && *err != ~0ull) return;  // a string failed the check: nothing is written
  for (uint32_t i = blockIdx.x * IO_W + wv; i < n; i += gridDim.x * IO_W) {  // wave-uniform
    if (apply && !apply[i]) continue;
    const uint8_t* s = data + off[i];
    const uint32_t slen = (uint32_t)(off[i + 1] - off[i]);
    const bool dense = s[4] == 0;
    if (!apply && dense) continue;  // nothing to check (exact length checked on the host)
    uint8_t* row = regs + ids[i] * HLL_REGS;
    const uint8_t* p = s + 16;
    const uint32_t plen = slen - 16;
    if (dense) {
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
    if (apply) {
      uint4* d4 = reinterpret_cast<uint4*>(S.row);
      for (uint32_t u = lane; u < HLL_REGS / 16; u += 64) d4[u] = make_uint4(0, 0, 0, 0);
      wave_lds_sync();
    }
    uint32_t at = 0, cin = 0;  // registers covered so far; byte 0 of the step is an XZERO second byte
    bool ok = true, can = true;
    for (uint32_t c0 = 0; c0 < plen; c0 += 64) {
      const uint32_t q = c0 + lane;
      const bool in = q < plen;
      const uint32_t b = in ? p[q] : 0u;
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
        const uint32_t b1 = q + 1 < plen ? p[q + 1] : 0u;
        run = sp_op(b, b1, &val, &two);
        if (two && q + 1 >= plen) ok = false;  // XZERO cut by the end of the string
        if (!apply) {
          // canonical form: the export's encoder would emit exactly this opcode here
          if (two && run <= 64) can = false;
          const uint32_t qn = q + (two ? 2 : 1);
          if (qn < plen) {
            uint32_t nv = 0;
            bool ntwo = false;
            (void)sp_op(p[qn], qn + 1 < plen ? p[qn + 1] : 0u, &nv, &ntwo);
            if (val == 0 && nv == 0) can = false;                  // two zero runs in a row
            if (val != 0 && nv == val && run < 4) can = false;     // a VAL run cut short
          }
        }
      }
      // register position of each opcode: exclusive prefix of the run lengths
      uint32_t x = run;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
      }
      const uint32_t first = at + x - run;
      if (apply && st && val != 0 && first + run <= (uint32_t)HLL_REGS)
        for (uint32_t r = 0; r < run; ++r) S.row[first + r] = (uint8_t)val;
      at += __shfl(x, 63, 64);
      if (at > (uint32_t)HLL_REGS) at = HLL_REGS + 1;  // (no wrap on adversarial input)
    }
    ok = __ballot(!ok) == 0 && at == (uint32_t)HLL_REGS;
    can = __ballot(!can) == 0;
    if (!apply) {
      if (lane == 0) {
        canon[i] = can ? 1 : 0;
        if (!ok) atomicMin(err, (unsigned long long)i);
      }
      continue;
    }
    wave_lds_sync();
    const uint4* s4 = reinterpret_cast<const uint4*>(S.row);
    for (uint32_t u = lane; u < HLL_REGS / 16; u += 64) reinterpret_cast<uint4*>(row)[u] = s4[u];
    if (lane == 0) card[ids[i]] = ld_u64(s + 8);
    wave_lds_sync();
  }
}

void hll_export_launch(rsk_ctx* c, const uint8_t* d_regs, const uint64_t* d_card, const uint64_t* d_ids,
                       const uint8_t* d_want_sparse, uint32_t n, uint32_t* d_len, uint8_t* d_slots) {
  if (!n) return;
  ProfScope ps(c, "hll_export_encode");
  const uint32_t blocks = std::min<uint32_t>((n + IO_W - 1) / IO_W, (uint32_t)c->num_cus * 4);
  hipLaunchKernelGGL(hll_export_kernel, dim3(blocks), dim3(IO_T), 0, c->stream, d_regs, d_card, d_ids, d_want_sparse,
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

void hll_import_launch(rsk_ctx* c, const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_ids,
                       const uint8_t* d_apply, uint32_t n, uint8_t* d_regs, uint64_t* d_card, uint8_t* d_canon,
                       unsigned long long* d_err) {
  if (!n) return;
  ProfScope ps(c, d_apply ? "hll_import_write" : "hll_import_check");
  const uint32_t blocks = std::min<uint32_t>((n + IO_W - 1) / IO_W, (uint32_t)c->num_cus * 4);
  hipLaunchKernelGGL(hll_import_kernel, dim3(blocks), dim3(IO_T), 0, c->stream, d_data, d_off, d_ids, d_apply, n,
                     d_regs, d_card, d_canon, d_err);
  RSK_CHECK_LAUNCH("hll_import");
}

}  // namespace rsk
