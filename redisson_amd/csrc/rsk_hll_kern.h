// rsk_hll_kern.h -- HLL PFADD kernels shared by librsketch (rsk_hll.hip,
// the production instantiations) and the test / bench support library
// (diag/rsk_diag_kernels.hip, the tuning variants of the same templates).
// Everything is in an anonymous namespace: each translation unit
// instantiates its own kernels.
#pragma once
#include "rsk_internal.h"

namespace rsk {
namespace {

// Byte-wise max of four 7-bit lanes (registers are <= 63).
RSK_DEV uint32_t bmax4(uint32_t a, uint32_t b) {
  uint32_t d = (a | 0x80808080u) - b;
  uint32_t m = ((d & 0x80808080u) >> 7) * 0xFFu;
  return (a & m) | (b & ~m);
}
RSK_DEV uint4 bmax16(uint4 a, uint4 b) {
  return make_uint4(bmax4(a.x, b.x), bmax4(a.y, b.y), bmax4(a.z, b.z), bmax4(a.w, b.w));
}

// ------------------------------------------------------------------ PFADD
__device__ __forceinline__ void lds_zero(uint32_t* regs) {
  uint4* r4 = reinterpret_cast<uint4*>(regs);
  for (int j = threadIdx.x; j < HLL_REGS / 4; j += blockDim.x) r4[j] = make_uint4(0, 0, 0, 0);
}

// Pack the LDS file (u32 per register) into 16384 bytes of the slab.
__device__ __forceinline__ void lds_to_slab(const uint32_t* regs, uint8_t* slab) {
  const uint4* r4 = reinterpret_cast<const uint4*>(regs);
  uint4* out = reinterpret_cast<uint4*>(slab);
  for (int j = threadIdx.x; j < HLL_REGS / 16; j += blockDim.x) {
    uint4 a = r4[4 * j], b = r4[4 * j + 1], c = r4[4 * j + 2], d = r4[4 * j + 3];
    uint4 o;
    o.x = a.x | (a.y << 8) | (a.z << 16) | (a.w << 24);
    o.y = b.x | (b.y << 8) | (b.z << 16) | (b.w << 24);
    o.z = c.x | (c.y << 8) | (c.z << 16) | (c.w << 24);
    o.w = d.x | (d.y << 8) | (d.z << 16) | (d.w << 24);
    out[j] = o;
  }
}

RSK_DEV void hll_update(uint32_t* regs, uint64_t h) {
  atomicMax(&regs[hll_index(h)], hll_rank(h));
}

// Fixed 16-byte keys: the C2 hot path.  U keys per lane in flight, T lanes
// per workgroup (256 measured fastest: fewer waves contend for the LDS file).
template <int U, int T>
__global__ __launch_bounds__(T) void hll_add16_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                      uint64_t per_block, uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs[HLL_REGS];
  lds_zero(regs);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  uint64_t i = begin + threadIdx.x;
  for (; i + (uint64_t)(U - 1) * T < end; i += (uint64_t)U * T) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld_nt16(&keys[i + (uint64_t)u * T]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t w0 = ((uint64_t)v[u].y << 32) | v[u].x;
      uint64_t w1 = ((uint64_t)v[u].w << 32) | v[u].z;
      hll_update(regs, murmur64a_16(w0, w1));
    }
  }
  for (; i < end; i += T) {
    uint4 v = keys[i];
    hll_update(regs, murmur64a_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z));
  }
  __syncthreads();
  lds_to_slab(regs, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

// ---- byte-register LDS file (16 KiB): check-then-CAS update.  After the
// first few keys per register almost every key only reads its register
// (a rank above the current value is rare), so the RMW is rarely taken and
// the 4x smaller file leaves LDS for staging and for more workgroups.
RSK_DEV void hll_update8(uint32_t* regs32, uint64_t h) {
  const uint32_t idx = hll_index(h), rank = hll_rank(h);
  uint32_t* w = regs32 + (idx >> 2);
  const uint32_t sh = (idx & 3u) * 8;
  uint32_t cur = *w;
  while (((cur >> sh) & 0xFFu) < rank) {
    const uint32_t nw = (cur & ~(0xFFu << sh)) | (rank << sh);
    const uint32_t prev = atomicCAS(w, cur, nw);
    if (prev == cur) break;
    cur = prev;
  }
}

// The same with the common case kept short (C4 is VALU-issue bound, see
// DESIGN.md): the rank from one 32-bit find-first-set of bits 14..45 (a
// rank above 32 -- those bits all zero -- takes the 64-bit form), one LDS
// read and compare; the CAS operands only on the rare path where the
// register grows.
RSK_DEV void hll_update8_fast(uint32_t* regs32, uint64_t h) {
  const uint32_t idx = (uint32_t)h & (HLL_REGS - 1);
  const uint32_t bits = (uint32_t)(h >> HLL_P);  // one v_alignbit
  uint32_t rank = 1u + (uint32_t)__builtin_ctz(bits | 0x80000000u);
  if (__builtin_expect(bits == 0, 0)) rank = hll_rank(h);
  uint32_t* w = regs32 + (idx >> 2);
  const uint32_t sh = (idx & 3u) * 8;
  uint32_t cur = *w;
  if (__builtin_expect(((cur >> sh) & 0xFFu) >= rank, 1)) return;
  do {
    const uint32_t nw = (cur & ~(0xFFu << sh)) | (rank << sh);
    const uint32_t prev = atomicCAS(w, cur, nw);
    if (prev == cur) break;
    cur = prev;
  } while (((cur >> sh) & 0xFFu) < rank);
}

__device__ __forceinline__ void lds8_zero(uint32_t* regs32) {
  uint4* r4 = reinterpret_cast<uint4*>(regs32);
  for (int j = threadIdx.x; j < HLL_REGS / 16; j += blockDim.x) r4[j] = make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ void lds8_to_slab(const uint32_t* regs32, uint8_t* slab) {
  const uint4* r4 = reinterpret_cast<const uint4*>(regs32);
  uint4* out = reinterpret_cast<uint4*>(slab);
  for (int j = threadIdx.x; j < HLL_REGS / 16; j += blockDim.x) out[j] = r4[j];
}

// Blob + offsets, LDS-staged (the C4 path).  A workgroup takes tiles of 512
// consecutive keys; their bytes are one contiguous blob range, copied into
// LDS with coalesced 16-byte loads that are issued one tile ahead (register
// prefetch; the tile's end offset is itself loaded a tile earlier, so the
// stage loads never wait on an offset load).  MurmurHash64A is a serial
// chain of ceil(len/8) multiply-bound steps and a wave runs as long as its
// longest key, so the tile's keys are counting-sorted by step count in LDS
// (one LDS atomic per key gives its rank in its class) and each lane then
// hashes KPL adjacent keys of that order, so the lanes of a wave see nearly
// equal lengths.  KPL = 1 in production (measured: KPL 2 and 4 interleave
// independent chains but lose more to registers and selects than they win,
// scripts/var_variants.py).  A tile whose bytes exceed the stage is hashed
// from global memory, unsorted.  The tile's barriers order LDS only
// (lds_barrier): __syncthreads' fence would wait for the next tile's stage
// loads at the first barrier after they are issued, undoing the prefetch.
constexpr int VAR_TILE = 512;                   // keys per tile
constexpr int VAR_STAGE = 32768;                // bytes per tile (64 B per key)
constexpr uint32_t VAR_MAXCLS = 16;             // step classes 0..16 (16 = that long or longer)
constexpr uint32_t VAR_NONE = VAR_MAXCLS + 1;   // slot past the end of the tile
constexpr int VAR_NCLS_PAD = 20;                // classes 0..17, padded

// One unaligned 8-byte LDS read (gfx950 LDS takes byte-aligned ds_read_b64;
// hipcc emits it for the memcpy).
RSK_DEV uint64_t lds_u64(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}

// MurmurHash64A of KPL keys of the stage (bytes [off, off+len)), as KPL
// interleaved chains over max(len/8) steps; a chain past its own blocks
// keeps its value (its clamped read stays inside its key + 7 bytes).  The
// tail read may run up to 7 bytes past a key, inside the stage's slack;
// those bytes are masked off.
// The loop runs ceil(len/8) - 1 full blocks and the last step is a select
// (the tail masked, or the last full block mixed): every key of one step
// class takes the same trip count, so a class-sorted wave does not pay the
// full loop + odd remainder + tail of its mixed nb = len >> 3 (measured form
// before: 5.8 step-times per wave on the C4 lengths 8..64 instead of 4.9).
RSK_DEV uint64_t murmur64a_lds(const uint8_t* p, uint32_t len) {
  const uint32_t steps = (len + 7) >> 3, t = len & 7;
  uint64_t h = (uint64_t)HLL_SEED ^ ((uint64_t)len * MM_M);
  if (steps) {
    for (uint32_t j = 0; j + 1 < steps; ++j) {
      h ^= mm_mix(lds_u64(p + 8 * j));
      h *= MM_M;
    }
    const uint64_t v = lds_u64(p + 8 * (steps - 1));
    const uint64_t x = t ? (v & ((1ULL << (8 * t)) - 1)) : mm_mix(v);
    h = (h ^ x) * MM_M;
  }
  return mm_final(h);
}
// Form 1 (form 2 is production: the same with aligned LDS reads): the loop runs the key's FULL blocks (len >> 3, the
// class the tile is sorted by) and the tail step (h ^= masked tail; h *= m)
// is computed for every key and kept by a select where len & 7 != 0.  Form 0
// above sorts by ceil(len/8) and ends in a branch between the masked tail
// and the mixed last block: every class holds one length with len & 7 == 0,
// so nearly every wave ran both sides (9 quarter-rate multiplies for its last
// step instead of 3).  h0 = HLL_SEED ^ len * m comes from a table.
RSK_DEV uint64_t murmur64a_lds_full(const uint8_t* p, uint32_t len, uint64_t h0) {
  const uint32_t nfull = len >> 3, t = len & 7;
  uint64_t h = h0;
  for (uint32_t j = 0; j < nfull; ++j) {
    h ^= mm_mix(lds_u64(p + 8 * j));
    h *= MM_M;
  }
  const uint64_t x = lds_u64(p + 8 * nfull) & ((1ULL << (8 * t)) - 1);  // t == 0: nothing (mask 0)
  const uint64_t ht = (h ^ x) * MM_M;
  h = t ? ht : h;
  return mm_final(h);
}

// Form 2: the same hash with only dword-aligned LDS reads.  The stage holds
// the blob verbatim, so a key starts at any byte; form 1's 8-byte reads at
// byte offsets (hipcc pairs them into ds_read_b128) are unaligned LDS
// accesses, and the C4 counters (profiles/r04_c4_sq.json) show the LDS
// stalled on them for about half of the kernel.  Here block j is assembled
// from the aligned dwords around it with one v_alignbit per 32 bits (shift =
// 8 x (offset mod 4)).
RSK_DEV uint32_t lds_dw(const uint32_t* w, uint32_t i) { return w[i]; }
RSK_DEV uint64_t murmur64a_lds_aligned(const uint8_t* p, uint32_t len, uint64_t h0) {
  const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p - (a & 3));
  const uint32_t s = (a & 3) * 8;
  const uint32_t nfull = len >> 3, t = len & 7;
  uint64_t h = h0;
  uint32_t v0 = lds_dw(w, 0);
  for (uint32_t j = 0; j < nfull; ++j) {
    const uint32_t v1 = lds_dw(w, 2 * j + 1), v2 = lds_dw(w, 2 * j + 2);
    const uint32_t lo = __builtin_amdgcn_alignbit(v1, v0, s), hi = __builtin_amdgcn_alignbit(v2, v1, s);
    h ^= mm_mix(((uint64_t)hi << 32) | lo);
    h *= MM_M;
    v0 = v2;
  }
  const uint32_t v1 = lds_dw(w, 2 * nfull + 1), v2 = lds_dw(w, 2 * nfull + 2);
  const uint64_t tail = ((uint64_t)__builtin_amdgcn_alignbit(v2, v1, s) << 32) | __builtin_amdgcn_alignbit(v1, v0, s);
  const uint64_t x = tail & ((1ULL << (8 * t)) - 1);  // t == 0: nothing (mask 0)
  const uint64_t ht = (h ^ x) * MM_M;
  h = t ? ht : h;
  return mm_final(h);
}

template <int KPL>
RSK_DEV void murmur64a_lds_multi(const uint8_t* st, const uint32_t (&off)[KPL], const uint32_t (&len)[KPL],
                                 uint64_t (&h)[KPL]) {
  if constexpr (KPL == 1) {
    h[0] = murmur64a_lds(st + off[0], len[0]);
    return;
  }
  uint32_t nb[KPL], nmax = 0;
#pragma unroll
  for (int q = 0; q < KPL; ++q) {
    nb[q] = len[q] >> 3;
    nmax = nb[q] > nmax ? nb[q] : nmax;
    h[q] = (uint64_t)HLL_SEED ^ ((uint64_t)len[q] * MM_M);
  }
  for (uint32_t j = 0; j < nmax; ++j) {
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const uint32_t jj = j < nb[q] ? j : nb[q];
      const uint64_t hn = (h[q] ^ mm_mix(lds_u64(st + off[q] + 8 * jj))) * MM_M;
      h[q] = j < nb[q] ? hn : h[q];
    }
  }
#pragma unroll
  for (int q = 0; q < KPL; ++q) {
    const uint32_t t = len[q] & 7;
    if (t) h[q] = (h[q] ^ (lds_u64(st + off[q] + 8 * nb[q]) & ((1ULL << (8 * t)) - 1))) * MM_M;
    h[q] = mm_final(h[q]);
  }
}

// Bytes [off, off+len) of the stage, or of global memory for an unstaged tile.
RSK_DEV uint64_t var_hash(bool staged, const uint64_t* st, uint32_t off, const uint8_t* g, uint64_t len) {
  if (staged) return murmur64a_lds(reinterpret_cast<const uint8_t*>(st) + off, (uint32_t)len);
  return len <= 64 ? murmur64a_le64(g, (uint32_t)len) : murmur64a(g, len);
}

// KPL keys per lane, 512 / KPL lanes; 3 workgroups per CU (LDS ~50 KiB each).
// DIAG (the support library's variants only): bit 0 replaces MurmurHash64A by one
// 8-byte read of the key, bit 1 skips the register update (XOR-folded into a
// slab byte instead): the cost of the rest of the kernel without them.
// F (form): 2 = production (full-block classes, select tail, h0 table,
// short register update, dword-aligned LDS reads); 1 = the same with 8-byte
// reads at byte offsets; 0 = the round-3 form (support library A/B only).
// STAGE: stage bytes per tile; OCC: workgroups per CU the launch bounds ask
// for (3 with the 32 KiB stage; 4 fit with 20 KiB -- 512 C4 keys span
// 18.4 KiB +- 0.4 -- and 64 VGPRs).
template <int KPL, int DIAG = 0, int F = 2, int STAGE = VAR_STAGE, int OCC = 3>
__global__ __launch_bounds__(VAR_TILE / KPL, OCC * VAR_TILE / KPL / 256) void hll_add_var_staged_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets, uint64_t n, uint64_t per_block,
    uint8_t* __restrict__ slabs) {
  constexpr int T = VAR_TILE / KPL;
  constexpr int PF = (STAGE / 16 + T - 1) / T;  // 16-byte stage chunks per lane
  constexpr bool FULL = F >= 1 && KPL == 1;  // F 1: unaligned 8-byte reads; F 2: aligned dwords
  __shared__ __attribute__((aligned(16))) uint32_t regs32[HLL_REGS / 4];
  __shared__ __attribute__((aligned(16))) uint64_t stage[STAGE / 8 + 4];
  __shared__ uint32_t perm[VAR_TILE];  // sorted keys: stage offset | len << 16
  __shared__ uint32_t cnt[VAR_NCLS_PAD], cbase[VAR_NCLS_PAD];
  __shared__ uint64_t h0tab[FULL ? 65 : 1];  // HLL_SEED ^ len * m, len <= 64
  const uint32_t tid = threadIdx.x;
  lds8_zero(regs32);
  if (tid < VAR_NCLS_PAD) cnt[tid] = 0;
  if constexpr (FULL)
    for (uint32_t j = tid; j <= 64; j += T) h0tab[j] = (uint64_t)HLL_SEED ^ ((uint64_t)j * MM_M);
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  const uintptr_t dbase = reinterpret_cast<uintptr_t>(data);
  const uint8_t* st8 = reinterpret_cast<const uint8_t*>(stage);
  uint64_t diag_acc = 0;

  // Tile state, one tile ahead.  The stage window starts at the 16-byte-
  // aligned ADDRESS at or below the tile's first byte, so no chunk load
  // crosses into a page the blob does not touch.  Lane key q is tile key
  // tid + q*T (coalesced offset loads).
  uint64_t last = 0, hi_ahead = 0, s[KPL], e[KPL];
  uintptr_t a0 = 0;
  uint32_t nchunk = 0;
  bool staged = false;
  uint4 pf[PF];
  auto fetch = [&](uint64_t b, uint64_t lo, uint64_t hi) {
    last = b + VAR_TILE < end ? b + VAR_TILE : end;
    a0 = (dbase + lo) & ~uintptr_t(15);
    const uint64_t span = dbase + hi - a0;
    staged = span <= (uint64_t)STAGE;
    nchunk = staged ? (uint32_t)((span + 15) >> 4) : 0;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const uint32_t c = tid + (uint32_t)u * T;
      // addressed from `data` (a global kernel argument), not from the integer
      // a0: a pointer rebuilt from an integer is generic, and its flat loads
      // count in lgkmcnt, so every LDS-only barrier of the tile would wait
      // for this prefetch
      if (c < nchunk) pf[u] = ld_nt16(reinterpret_cast<const uint4*>(data + (a0 - dbase)) + c);
    }
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const uint64_t i = b + tid + (uint64_t)q * T;
      s[q] = i < last ? offsets[i] : 0;
      e[q] = i < last ? offsets[i + 1] : 0;
    }
    hi_ahead = offsets[last + VAR_TILE < end ? last + VAR_TILE : end];  // the following tile's end
  };
  uint64_t cur_hi = 0;
  if (begin < end) {
    cur_hi = offsets[begin + VAR_TILE < end ? begin + VAR_TILE : end];
    fetch(begin, offsets[begin], cur_hi);
  }

  for (uint64_t base = begin; base < end;) {
    lds_barrier();  // [A] previous tile's stage / perm / cbase reads are done
    uint4* st16 = reinterpret_cast<uint4*>(stage);
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const uint32_t c = tid + (uint32_t)u * T;
      if (c < nchunk) st16[c] = pf[u];
    }
    const bool cur_staged = staged;  // workgroup-uniform
    uint32_t cls[KPL], rk[KPL], coff[KPL];
    uint64_t clen[KPL], cs[KPL];
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const bool mine = base + tid + (uint64_t)q * T < last;
      clen[q] = e[q] - s[q];
      cs[q] = s[q];
      coff[q] = (uint32_t)(dbase + s[q] - a0);
      const uint64_t steps = FULL ? clen[q] >> 3 : (clen[q] + 7) >> 3;  // the hash loop's trip count
      cls[q] = !mine ? VAR_NONE : (steps < VAR_MAXCLS ? (uint32_t)steps : VAR_MAXCLS);
      rk[q] = (cur_staged && cls[q] != VAR_NONE) ? atomicAdd(&cnt[cls[q]], 1u) : 0u;  // rank inside the class
    }
    // Issue the next tile's loads (they land while this tile hashes).
    const uint64_t next = last;
    if (next < end) {
      const uint64_t lo_n = cur_hi;
      cur_hi = hi_ahead;
      fetch(next, lo_n, cur_hi);
    }
    lds_barrier();  // [B] stage written, class counts final
    if (cur_staged) {
      if (tid < 64) {  // class starts: wave 0's exclusive prefix over the counts (one LDS read per lane)
        const uint32_t v = tid < VAR_NCLS_PAD ? cnt[tid] : 0;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const uint32_t y = __shfl_up(x, o, 64);
          if (tid >= (uint32_t)o) x += y;
        }
        if (tid < VAR_NCLS_PAD) cbase[tid] = x - v;
      }
      lds_barrier();  // [C]
#pragma unroll
      for (int q = 0; q < KPL; ++q)
        if (cls[q] != VAR_NONE) perm[cbase[cls[q]] + rk[q]] = coff[q] | ((uint32_t)clen[q] << 16);
      lds_barrier();  // [D]
      if (tid < VAR_NCLS_PAD) cnt[tid] = 0;
      const uint32_t nvalid = cbase[VAR_NONE];
      uint32_t o[KPL], l[KPL], pos[KPL];
#pragma unroll
      for (int q = 0; q < KPL; ++q) {
        // adjacent sorted keys: one class per lane, nearly.  With one key per
        // lane, wave w takes sorted chunk w (w < 4) or 11 - w, so the two waves
        // a SIMD holds (w, w + 4) get a short and a long chunk: the SIMDs
        // finish a tile together instead of the one with the longest keys
        // holding the workgroup at the next barrier.
        if constexpr (KPL == 1 && T == 512) {
          const uint32_t w = tid >> 6;
          pos[q] = (w < 4 ? w : 11 - w) * 64 + (tid & 63);
        } else {
          pos[q] = tid * KPL + q;
        }
        const uint32_t p = pos[q] < nvalid ? perm[pos[q]] : 0u;
        o[q] = p & 0xFFFFu;
        l[q] = p >> 16;
      }
      uint64_t h[KPL];
      if constexpr (DIAG & 1) {
#pragma unroll
        for (int q = 0; q < KPL; ++q) h[q] = lds_u64(st8 + o[q]) ^ l[q];
      } else if constexpr (FULL) {
        uint64_t h0 = h0tab[l[0] <= 64 ? l[0] : 0];
        if (l[0] > 64) h0 = (uint64_t)HLL_SEED ^ ((uint64_t)l[0] * MM_M);
        h[0] = F == 2 ? murmur64a_lds_aligned(st8 + o[0], l[0], h0) : murmur64a_lds_full(st8 + o[0], l[0], h0);
      } else {
        murmur64a_lds_multi<KPL>(st8, o, l, h);
      }
#pragma unroll
      for (int q = 0; q < KPL; ++q)
        if (pos[q] < nvalid) {
          if constexpr (DIAG & 2) diag_acc ^= h[q];
          else if constexpr (FULL) hll_update8_fast(regs32, h[q]);
          else hll_update8(regs32, h[q]);
        }
    } else {
#pragma unroll
      for (int q = 0; q < KPL; ++q)
        if (cls[q] != VAR_NONE) {
          if constexpr (FULL) hll_update8_fast(regs32, var_hash(false, stage, 0, data + cs[q], clen[q]));
          else hll_update8(regs32, var_hash(false, stage, 0, data + cs[q], clen[q]));
        }
    }
    base = next;
  }
  __syncthreads();
  lds8_to_slab(regs32, slabs + (uint64_t)blockIdx.x * HLL_REGS);
  if constexpr ((DIAG & 2) != 0) slabs[(uint64_t)blockIdx.x * HLL_REGS + tid] = (uint8_t)(diag_acc % 51);
}

// ---- The ring form (a support-library experiment, not routed: C4 11.3 ms
// against 9.4 for form 2, profiles/r04_c4_sq.json).
// The stage of a tile is filled by LDS-DMA (global_load_lds_dwordx4: no
// VGPRs) into a ring of three 20 KiB slots, TWO tiles ahead, and the tile's
// key offsets are loaded a tile ahead; the waits are counted (vmcnt) and the
// barriers raw, so the two stages in flight stay in flight across the tile's
// barriers.  Round 3's form held one tile ahead in registers: with the hash
// between two tiles the stream ran at 4.5 TB/s (the same kernel without the
// hash: 6.5), i.e. too few bytes in flight per CU.  The LDS-DMA and the
// offset loads are issued from inline asm so the compiler neither inserts a
// vmcnt(0) before every LDS read (its LDS-DMA alias tracking) nor counts
// them; every wait for them below is explicit.  Classes, hash and register
// update are form 1's.  2 workgroups per CU (LDS ~79 KiB each).
constexpr uint32_t RING_SLOTS = 3;
constexpr uint32_t RING_SB = 20480;           // stage bytes per slot (512 C4 keys: 18.4 KiB +- 0.4)
constexpr uint32_t RING_CH = RING_SB / 16;    // 1280 16-byte chunks: waves 0-3 load 3 per lane, 4-7 load 2
constexpr uint32_t RING_MAX_MEAN = 37;        // host route: mean key bytes for which a tile fits a slot

// One LDS-DMA of 16 bytes per lane: lane i writes LDS [base + 16 i, +16) from
// gptr (per lane); base is wave-uniform (M0).  Not visible to the compiler's
// wait counting: the caller waits with ring_wait.
RSK_DEV void ring_glds16(const void* gptr, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds_base), "v"(gptr)
               : "memory");
}
// A u64 load the compiler does not count (the caller waits with ring_wait
// and passes the value through ring_ready before using it).
RSK_DEV uint64_t ring_ld64(const uint64_t* p) {
  uint64_t v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}
// A wave-uniform u64 by a scalar load (lgkmcnt; never a vmcnt wait that
// would retire the stages in flight).
RSK_DEV uint64_t ring_sld64(const uint64_t* p) {
  uint64_t v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p));
  return v;
}
RSK_DEV void ring_ready(uint64_t& a, uint64_t& b) { asm volatile("" : "+v"(a), "+v"(b)); }

template <int DIAG = 0>
__global__ __launch_bounds__(VAR_TILE, 2) void hll_add_var_ring_kernel(const uint8_t* __restrict__ data,
                                                                      const uint64_t* __restrict__ offsets,
                                                                      uint64_t n, uint64_t per_block,
                                                                      uint8_t* __restrict__ slabs) {
  constexpr uint32_t T = VAR_TILE;
  __shared__ __attribute__((aligned(16))) uint32_t regs32[HLL_REGS / 4];
  __shared__ __attribute__((aligned(16))) uint4 ring[RING_SLOTS * RING_CH + 2];  // + slack: tail reads past a span
  __shared__ uint32_t perm[VAR_TILE];
  __shared__ uint32_t cnt[VAR_NCLS_PAD], cbase[VAR_NCLS_PAD];
  __shared__ uint64_t h0tab[65];
  const uint32_t tid = threadIdx.x, wv = tid >> 6;
  const uint32_t nld = wv < 4 ? 3u : 2u;  // this wave's LDS-DMA per tile (1280 chunks)
  lds8_zero(regs32);
  if (tid < VAR_NCLS_PAD) cnt[tid] = 0;
  for (uint32_t j = tid; j <= 64; j += T) h0tab[j] = (uint64_t)HLL_SEED ^ ((uint64_t)j * MM_M);
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  const uintptr_t dbase = reinterpret_cast<uintptr_t>(data);
  const uint32_t ring_lds = (uint32_t)reinterpret_cast<uintptr_t>(ring);

  // Tile t covers keys [begin + tT, min(begin + (t+1)T, end)); its bytes are
  // blob [H(t-1), H(t)) with H(t) = offsets[min(begin + (t+1)T, end)] and
  // H(-1) = offsets[begin].  The window of a tile: a0 (the 16-byte-aligned
  // address at or below its first byte), whether its span fits a slot, and
  // its 16-byte chunk count.  At tile t the H values up to H(t+2) are at
  // hand: H(t+3) is scalar-loaded at tile t and waited for at its end (its
  // latency hides behind the tile), so no scalar load stalls the loop.
  auto hidx = [&](uint64_t t) {  // offsets index of H(t), t >= -1 (as uint64: t + 1)
    const uint64_t k = begin + t * T;
    return k < end ? k : end;
  };
  auto wnd = [&](uint64_t lo, uint64_t hi, uintptr_t* a0, bool* fits) {
    *a0 = (dbase + lo) & ~uintptr_t(15);
    *fits = dbase + hi - *a0 <= RING_SB;
    return (uint32_t)((dbase + hi - *a0 + 15) >> 4);
  };
  // LDS-DMA of the tile with bytes [lo, hi) into slot `slot` (every wave
  // issues exactly nld DMAs whatever the tile: chunks past the window re-read
  // its last chunk; a tile past the range, unstaged or of no bytes reads the
  // offsets array -- valid memory -- into the slot, which nobody reads then).
  auto issue = [&](bool valid, uint64_t lo, uint64_t hi, uint32_t slot) {
    const uint8_t* src0 = reinterpret_cast<const uint8_t*>(offsets);
    uint32_t nch = 1;
    if (valid) {
      uintptr_t a0;
      bool fits;
      const uint32_t k = wnd(lo, hi, &a0, &fits);
      if (fits && k > 0) {
        src0 = data + (a0 - dbase);
        nch = k;
      }
    }
    for (uint32_t u = 0; u < nld; ++u) {
      const uint32_t c = tid + u * T;
      const uint32_t cc = c < nch ? c : nch - 1;
      ring_glds16(src0 + 16 * (uint64_t)cc,
                  __builtin_amdgcn_readfirstlane(ring_lds + 16 * (slot * RING_CH + u * T + wv * 64)));
    }
  };
  // Everything this wave issued before its newest nld DMAs has landed.  Issue
  // order per tile is [H(t+3)], [next tile's key offsets], then [stage two
  // tiles ahead], so this retires H(t+3), the key offsets and the stage of
  // the next tile (issued a tile earlier) and leaves the farthest stage in
  // flight.
  auto wait_ring = [&] {
    if (wv < 4) asm volatile("s_waitcnt vmcnt(3)");
    else asm volatile("s_waitcnt vmcnt(2)");
  };
  auto key_offsets = [&](uint64_t b, uint64_t* s, uint64_t* e) {
    const uint64_t i = b + tid < n ? b + tid : n - 1;  // lanes past the batch: valid, unused
    *s = ring_ld64(offsets + i);
    *e = ring_ld64(offsets + i + 1);
  };

  if (begin >= end) {  // nothing to do (a workgroup past the batch)
    __syncthreads();
    lds8_to_slab(regs32, slabs + (uint64_t)blockIdx.x * HLL_REGS);
    return;
  }
  // prologue: H(-1..2), key offsets of tile 0, stages of tiles 0 and 1
  uint64_t Hm = ring_sld64(offsets + begin);
  uint64_t H0 = ring_sld64(offsets + hidx(1));
  uint64_t H1 = ring_sld64(offsets + hidx(2));
  uint64_t H2 = ring_sld64(offsets + hidx(3));
  uint64_t s_cur = 0, e_cur = 0, s_nxt = 0, e_nxt = 0;
  key_offsets(begin, &s_cur, &e_cur);
  issue(true, Hm, H0, 0);
  issue(begin + T < end, H0, H1, 1);
  wait_ring();  // offsets 0 and stage 0 (issued before stage 1)
  ring_ready(s_cur, e_cur);
  uint32_t slot = 0;
  uint64_t t = 0;
  for (uint64_t base = begin; base < end; base += T, ++t) {
    lds_barrier();  // [A] every wave's DMAs of this tile's stage landed; last tile's stage / perm reads done
    const uint64_t last = base + T < end ? base + T : end;
    uintptr_t a0;
    bool fits;
    (void)wnd(Hm, H0, &a0, &fits);
    // issue: H(t+3), next tile's key offsets, the stage two tiles ahead.  H(t+3)
    // is a vector load of one address (a scalar load would be retired by the
    // lgkmcnt(0) of the next LDS barrier, a stall of its full latency).
    uint64_t H3v = ring_ld64(offsets + hidx(t + 4));
    if (base + T < end) key_offsets(base + T, &s_nxt, &e_nxt);
    issue(base + 2 * T < end, H1, H2, (slot + 2) % RING_SLOTS);
    const bool mine = base + tid < last;
    const uint64_t clen = e_cur - s_cur;
    const uint32_t coff = (uint32_t)(dbase + s_cur - a0);
    const uint64_t nfull = clen >> 3;
    const uint32_t cls = !mine ? VAR_NONE : (nfull < VAR_MAXCLS ? (uint32_t)nfull : VAR_MAXCLS);
    const uint32_t rk = (fits && cls != VAR_NONE) ? atomicAdd(&cnt[cls], 1u) : 0u;
    lds_barrier();  // [B] class counts final
    const uint8_t* st8 = reinterpret_cast<const uint8_t*>(ring + slot * RING_CH);
    if (fits) {
      if (tid < 64) {
        const uint32_t v = tid < VAR_NCLS_PAD ? cnt[tid] : 0;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const uint32_t y = __shfl_up(x, o, 64);
          if (tid >= (uint32_t)o) x += y;
        }
        if (tid < VAR_NCLS_PAD) cbase[tid] = x - v;
      }
      lds_barrier();  // [C]
      if (cls != VAR_NONE) perm[cbase[cls] + rk] = coff | ((uint32_t)clen << 16);
      lds_barrier();  // [D]
      if (tid < VAR_NCLS_PAD) cnt[tid] = 0;
      const uint32_t nvalid = cbase[VAR_NONE];
      const uint32_t pos = (wv < 4 ? wv : 11 - wv) * 64 + (tid & 63);  // SIMD-balanced sorted chunks
      const uint32_t p = pos < nvalid ? perm[pos] : 0u;
      const uint32_t o = p & 0xFFFFu, l = p >> 16;
      uint64_t h0 = h0tab[l <= 64 ? l : 0];
      if (l > 64) h0 = (uint64_t)HLL_SEED ^ ((uint64_t)l * MM_M);
      uint64_t h;
      if constexpr (DIAG & 1) h = lds_u64(st8 + o) ^ h0;  // support library: the kernel without MurmurHash64A
      else h = murmur64a_lds_full(st8 + o, l, h0);
      if (pos < nvalid) hll_update8_fast(regs32, h);
    } else if (mine) {  // a tile whose bytes exceed a slot: hashed from global memory, unsorted
      hll_update8_fast(regs32, var_hash(false, nullptr, 0, data + s_cur, clen));
    }
    wait_ring();  // H(t+3), the next tile's key offsets and stage (this wave's part) landed
    ring_ready(s_nxt, e_nxt);
    asm volatile("" : "+v"(H3v));
    const uint64_t H3 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(H3v >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)H3v);
    s_cur = s_nxt;
    e_cur = e_nxt;
    Hm = H0;
    H0 = H1;
    H1 = H2;
    H2 = H3;
    slot = slot + 1 == RING_SLOTS ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
  __syncthreads();
  lds8_to_slab(regs32, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

inline void var_grid(rsk_ctx* c, uint64_t n, uint64_t* blocks, uint64_t* per_block, uint32_t occ = 3) {
  // LDS-staged tiles: ~50 KiB of LDS per workgroup -> 3 workgroups per CU (occ).
  uint64_t b = std::min<uint64_t>((n + VAR_TILE - 1) / VAR_TILE, std::min<uint64_t>(occ * (uint64_t)c->num_cus, c->slab_count));
  if (b == 0) b = 1;
  uint64_t pb = (n + b - 1) / b;
  pb = (pb + VAR_TILE - 1) / VAR_TILE * VAR_TILE;
  *per_block = pb;
  *blocks = (n + pb - 1) / pb;
}

}  // namespace
}  // namespace rsk
