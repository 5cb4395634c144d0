// rsk_hll.hip -- HyperLogLog kernels for gfx950 (Redis 3.2.0 semantics).
//
// Replaces the PFADD / PFCOUNT / PFMERGE arithmetic that RedissonHyperLogLog
// (src/main/java/org/redisson/RedissonHyperLogLog.java:65-97) delegates to the
// Redis server (hyperloglog.c: hllAdd/hllPatLen, hllCount, pfmergeCommand).
//
// Data layout in HBM: a pool of sketches, [n][16384] raw registers, one byte
// each (Redis's internal HLL_RAW form); the 6-bit dense packing only exists
// at the Redis export/import boundary.  Each pool also keeps card[n], the
// 8-byte cardinality cache of the Redis header.
//
// PFADD (streaming, HBM-bound): a persistent grid of 2 workgroups per CU.
// Every workgroup owns a private 16384 x u32 register file in LDS (64 KiB,
// so two fit in the CU's 160 KiB), streams a contiguous slice of the key
// array with 16-byte loads, hashes each key and applies ds_max_u32.  At the
// end it writes its file as 16 KiB of bytes (a "slab"); one reduce kernel
// max-merges all slabs and the sketch's old registers (deterministic, no
// global atomics), and raises a flag if any register grew.
#include <hipcub/hipcub.hpp>

#include "rsk_hllcount.h"
#include "rsk_internal.h"

namespace rsk {

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

// Tuning variants of the 16-byte kernel (rsk_diag_hll_variant): keys in
// flight per lane U, workgroup size T, nontemporal loads NT.
template <int U, int T, bool NT>
__global__ __launch_bounds__(T) void hll_add16_variant(const uint4* __restrict__ keys, uint64_t n, uint64_t per_block,
                                                       uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs[HLL_REGS];
  lds_zero(regs);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  uint64_t i = begin + threadIdx.x;
  for (; i + (uint64_t)(U - 1) * T < end; i += (uint64_t)U * T) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? ld_nt16(&keys[i + (uint64_t)u * T]) : keys[i + (uint64_t)u * T];
#pragma unroll
    for (int u = 0; u < U; ++u)
      hll_update(regs, murmur64a_16(((uint64_t)v[u].y << 32) | v[u].x, ((uint64_t)v[u].w << 32) | v[u].z));
  }
  for (; i < end; i += T) {
    uint4 v = keys[i];
    hll_update(regs, murmur64a_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z));
  }
  __syncthreads();
  lds_to_slab(regs, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

template <int U, int T, bool NT>
static void launch_variant(rsk_ctx* c, const uint4* keys, uint64_t n, uint32_t wg_per_cu) {
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * wg_per_cu, c->slab_count);
  const uint64_t tile = (uint64_t)T * U;
  uint64_t per_block = (n + blocks - 1) / blocks;
  per_block = (per_block + tile - 1) / tile * tile;
  blocks = (n + per_block - 1) / per_block;
  hipLaunchKernelGGL((hll_add16_variant<U, T, NT>), dim3((uint32_t)blocks), dim3(T), 0, c->stream, keys, n, per_block,
                     c->d_slab);
}

// Software-pipelined variant: the next U keys per lane load while the
// current U are hashed (no stores in the loop, so the in-order vmcnt lets
// the wait cover only the older loads).
template <int U, int T>
__global__ __launch_bounds__(T) void hll_add16_pf(const uint4* __restrict__ keys, uint64_t n, uint64_t per_block,
                                                  uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs[HLL_REGS];
  lds_zero(regs);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  uint64_t i = begin + threadIdx.x;
  uint4 v[U];
  if (i + (uint64_t)(U - 1) * T < end) {
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld_nt16(&keys[i + (uint64_t)u * T]);
  }
  for (; i + (uint64_t)(U - 1) * T < end; i += (uint64_t)U * T) {
    uint4 cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = v[u];
    const uint64_t j = i + (uint64_t)U * T;
    if (j + (uint64_t)(U - 1) * T < end) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld_nt16(&keys[j + (uint64_t)u * T]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      hll_update(regs, murmur64a_16(((uint64_t)cur[u].y << 32) | cur[u].x, ((uint64_t)cur[u].w << 32) | cur[u].z));
  }
  for (; i < end; i += T) {
    uint4 x = keys[i];
    hll_update(regs, murmur64a_16(((uint64_t)x.y << 32) | x.x, ((uint64_t)x.w << 32) | x.z));
  }
  __syncthreads();
  lds_to_slab(regs, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

template <int U, int T>
static void launch_pf(rsk_ctx* c, const uint4* keys, uint64_t n) {
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * 2, c->slab_count);
  const uint64_t tile = (uint64_t)T * U;
  uint64_t per_block = (n + blocks - 1) / blocks;
  per_block = (per_block + tile - 1) / tile * tile;
  blocks = (n + per_block - 1) / per_block;
  hipLaunchKernelGGL((hll_add16_pf<U, T>), dim3((uint32_t)blocks), dim3(T), 0, c->stream, keys, n, per_block, c->d_slab);
}

template <int U, int T>
static void launch_b8(rsk_ctx* c, const uint4* keys, uint64_t n, uint32_t wg_per_cu);

void hll_variant_launch(rsk_ctx* c, int variant, const uint4* keys, uint64_t n) {
  switch (variant) {
    case 8: launch_b8<4, 512>(c, keys, n, 4); break;
    case 9: launch_b8<4, 256>(c, keys, n, 8); break;
    case 10: launch_b8<8, 512>(c, keys, n, 4); break;
    case 11: launch_b8<4, 1024>(c, keys, n, 2); break;
    case 12: launch_pf<4, 256>(c, keys, n); break;
    case 13: launch_pf<2, 256>(c, keys, n); break;
    case 14: launch_pf<8, 256>(c, keys, n); break;
    case 0: launch_variant<4, 512, true>(c, keys, n, 2); break;
    case 1: launch_variant<8, 512, true>(c, keys, n, 2); break;
    case 2: launch_variant<2, 512, true>(c, keys, n, 2); break;
    case 3: launch_variant<4, 512, false>(c, keys, n, 2); break;
    case 4: launch_variant<4, 1024, true>(c, keys, n, 2); break;
    case 5: launch_variant<4, 256, true>(c, keys, n, 2); break;
    case 6: launch_variant<8, 1024, true>(c, keys, n, 2); break;
    case 7: launch_variant<2, 1024, true>(c, keys, n, 2); break;
    default: throw RskError{RSK_ERR_INVALID_ARG, "unknown variant"};
  }
  RSK_CHECK_LAUNCH("hll_variant");
}

// Any fixed stride or blob+offsets: lane-per-key MurmurHash64A.
template <bool VAR>
__global__ __launch_bounds__(RSK_ADD_THREADS, 2) void hll_add_bytes_kernel(const uint8_t* __restrict__ data,
                                                                           const uint64_t* __restrict__ offsets,
                                                                           uint32_t fixed_len, uint64_t n,
                                                                           uint64_t per_block,
                                                                           uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs[HLL_REGS];
  lds_zero(regs);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  for (uint64_t i = begin + threadIdx.x; i < end; i += blockDim.x) {
    uint64_t s, len;
    if (VAR) {
      s = offsets[i];
      len = offsets[i + 1] - s;
    } else {
      s = i * fixed_len;
      len = fixed_len;
    }
    hll_update(regs, len <= 64 ? murmur64a_le64(data + s, (uint32_t)len) : murmur64a(data + s, len));
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

__device__ __forceinline__ void lds8_zero(uint32_t* regs32) {
  uint4* r4 = reinterpret_cast<uint4*>(regs32);
  for (int j = threadIdx.x; j < HLL_REGS / 16; j += blockDim.x) r4[j] = make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ void lds8_to_slab(const uint32_t* regs32, uint8_t* slab) {
  const uint4* r4 = reinterpret_cast<const uint4*>(regs32);
  uint4* out = reinterpret_cast<uint4*>(slab);
  for (int j = threadIdx.x; j < HLL_REGS / 16; j += blockDim.x) out[j] = r4[j];
}

// 16-byte keys with the byte-register file (tuning variant).
template <int U, int T>
__global__ __launch_bounds__(T) void hll_add16_b8_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                         uint64_t per_block, uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs32[HLL_REGS / 4];
  lds8_zero(regs32);
  __syncthreads();
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  uint64_t i = begin + threadIdx.x;
  for (; i + (uint64_t)(U - 1) * T < end; i += (uint64_t)U * T) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld_nt16(&keys[i + (uint64_t)u * T]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      hll_update8(regs32, murmur64a_16(((uint64_t)v[u].y << 32) | v[u].x, ((uint64_t)v[u].w << 32) | v[u].z));
  }
  for (; i < end; i += T) {
    uint4 v = keys[i];
    hll_update8(regs32, murmur64a_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z));
  }
  __syncthreads();
  lds8_to_slab(regs32, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

template <int U, int T>
static void launch_b8(rsk_ctx* c, const uint4* keys, uint64_t n, uint32_t wg_per_cu) {
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * wg_per_cu, c->slab_count);
  const uint64_t tile = (uint64_t)T * U;
  uint64_t per_block = (n + blocks - 1) / blocks;
  per_block = (per_block + tile - 1) / tile * tile;
  blocks = (n + per_block - 1) / per_block;
  hipLaunchKernelGGL((hll_add16_b8_kernel<U, T>), dim3((uint32_t)blocks), dim3(T), 0, c->stream, keys, n, per_block,
                     c->d_slab);
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
// DIAG (rsk_diag_hll_var_variant only): bit 0 replaces MurmurHash64A by one
// 8-byte read of the key, bit 1 skips the register update (XOR-folded into a
// slab byte instead): the cost of the rest of the kernel without them.
template <int KPL, int DIAG = 0>
__global__ __launch_bounds__(VAR_TILE / KPL, 3 * VAR_TILE / KPL / 256) void hll_add_var_staged_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets, uint64_t n, uint64_t per_block,
    uint8_t* __restrict__ slabs) {
  constexpr int T = VAR_TILE / KPL;
  constexpr int PF = VAR_STAGE / 16 / T;  // 16-byte stage chunks per lane
  __shared__ __attribute__((aligned(16))) uint32_t regs32[HLL_REGS / 4];
  __shared__ __attribute__((aligned(16))) uint64_t stage[VAR_STAGE / 8 + 4];
  __shared__ uint32_t perm[VAR_TILE];  // sorted keys: stage offset | len << 16
  __shared__ uint32_t cnt[VAR_NCLS_PAD], cbase[VAR_NCLS_PAD];
  const uint32_t tid = threadIdx.x;
  lds8_zero(regs32);
  if (tid < VAR_NCLS_PAD) cnt[tid] = 0;
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
    staged = span <= (uint64_t)VAR_STAGE;
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
      const uint64_t steps = (clen[q] + 7) >> 3;
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
      } else {
        murmur64a_lds_multi<KPL>(st8, o, l, h);
      }
#pragma unroll
      for (int q = 0; q < KPL; ++q)
        if (pos[q] < nvalid) {
          if constexpr (DIAG & 2) diag_acc ^= h[q];
          else hll_update8(regs32, h[q]);
        }
    } else {
#pragma unroll
      for (int q = 0; q < KPL; ++q)
        if (cls[q] != VAR_NONE) hll_update8(regs32, var_hash(false, stage, 0, data + cs[q], clen[q]));
    }
    base = next;
  }
  __syncthreads();
  lds8_to_slab(regs32, slabs + (uint64_t)blockIdx.x * HLL_REGS);
  if constexpr ((DIAG & 2) != 0) slabs[(uint64_t)blockIdx.x * HLL_REGS + tid] = (uint8_t)(diag_acc % 51);
}

// The round-1 form (no prefetch, no sort): the A/B baseline of the diag.
constexpr int VAR_T = 512;
__global__ __launch_bounds__(VAR_T) void hll_add_var_simple_kernel(const uint8_t* __restrict__ data,
                                                                   const uint64_t* __restrict__ offsets, uint64_t n,
                                                                   uint64_t per_block, uint8_t* __restrict__ slabs) {
  __shared__ __attribute__((aligned(16))) uint32_t regs32[HLL_REGS / 4];
  __shared__ __attribute__((aligned(16))) uint64_t stage[VAR_STAGE / 8 + 4];
  lds8_zero(regs32);
  const uint64_t begin = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = begin + per_block < n ? begin + per_block : n;
  const uintptr_t dbase = reinterpret_cast<uintptr_t>(data);
  for (uint64_t base = begin; base < end; base += VAR_T) {
    const uint64_t last = base + VAR_T < end ? base + VAR_T : end;
    const uint64_t i = base + threadIdx.x;
    const bool mine = i < last;
    const uint64_t s = mine ? offsets[i] : 0;
    const uint64_t e = mine ? offsets[i + 1] : 0;
    const uintptr_t a0 = (dbase + offsets[base]) & ~uintptr_t(15);
    const uint64_t span = dbase + offsets[last] - a0;
    const bool staged = span <= (uint64_t)VAR_STAGE;
    __syncthreads();  // previous tile's stage reads are done
    if (staged) {
      const uint32_t nchunk = (uint32_t)((span + 15) >> 4);
      const uint4* src = reinterpret_cast<const uint4*>(data + (a0 - dbase));
      uint4* dst = reinterpret_cast<uint4*>(stage);
      for (uint32_t c = threadIdx.x; c < nchunk; c += VAR_T) dst[c] = ld_nt16(src + c);
    }
    __syncthreads();
    if (mine) hll_update8(regs32, var_hash(staged, stage, (uint32_t)(dbase + s - a0), data + s, e - s));
  }
  __syncthreads();
  lds8_to_slab(regs32, slabs + (uint64_t)blockIdx.x * HLL_REGS);
}

static void var_grid(rsk_ctx* c, uint64_t n, uint64_t* blocks, uint64_t* per_block) {
  // LDS-staged tiles: ~50 KiB of LDS per workgroup -> 3 workgroups per CU.
  uint64_t b = std::min<uint64_t>((n + VAR_TILE - 1) / VAR_TILE, std::min<uint64_t>(3ull * c->num_cus, c->slab_count));
  if (b == 0) b = 1;
  uint64_t pb = (n + b - 1) / b;
  pb = (pb + VAR_TILE - 1) / VAR_TILE * VAR_TILE;
  *per_block = pb;
  *blocks = (n + pb - 1) / pb;
}

void hll_var_variant_launch(rsk_ctx* c, int variant, const uint8_t* data, const uint64_t* offsets, uint64_t n) {
  uint64_t blocks, per_block;
  var_grid(c, n, &blocks, &per_block);
  const dim3 g((uint32_t)blocks);
  switch (variant) {
    case 0: hipLaunchKernelGGL(hll_add_var_staged_kernel<1>, g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 1: hipLaunchKernelGGL(hll_add_var_staged_kernel<2>, g, dim3(VAR_TILE / 2), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 2: hipLaunchKernelGGL(hll_add_var_simple_kernel, g, dim3(VAR_T), 0, c->stream, data, offsets, n, per_block,
                               c->d_slab); break;
    case 3: hipLaunchKernelGGL(hll_add_var_staged_kernel<4>, g, dim3(VAR_TILE / 4), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 4: hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 1>), g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 5: hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 2>), g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    case 6: hipLaunchKernelGGL((hll_add_var_staged_kernel<1, 3>), g, dim3(VAR_TILE), 0, c->stream, data, offsets, n,
                               per_block, c->d_slab); break;
    default: throw RskError{RSK_ERR_INVALID_ARG, "unknown variant"};
  }
  RSK_CHECK_LAUNCH("hll_var_variant");
}

// Max-merge `nslabs` slabs and the sketch's registers; 64 registers per
// workgroup of 256 lanes (grid 256).  If any register grew: *flag =
// max(*flag, epoch) (the caller's call number, so no reset is needed) and
// the Redis card cache is invalidated (HLL_INVALIDATE_CACHE), as it is when
// the key was just created.
__global__ __launch_bounds__(256) void hll_reduce_kernel(const uint8_t* __restrict__ slabs, uint32_t nslabs,
                                                         uint8_t* __restrict__ regs, uint32_t* __restrict__ flag,
                                                         uint32_t epoch, unsigned long long* __restrict__ card,
                                                         int created) {
  if (created && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(card, 1ull << 63);
  __shared__ uint4 part[4][256];
  const int t = threadIdx.x;
  const uint64_t col = (uint64_t)blockIdx.x * 64;  // first register of this block
  uint4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = make_uint4(0, 0, 0, 0);
  for (uint32_t s = t; s < nslabs; s += 256) {
    const uint4* p = reinterpret_cast<const uint4*>(slabs + (uint64_t)s * HLL_REGS + col);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = bmax16(acc[q], p[q]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) part[q][t] = acc[q];
  __syncthreads();
  for (int stride = 128; stride > 0; stride >>= 1) {
    if (t < stride) {
#pragma unroll
      for (int q = 0; q < 4; ++q) part[q][t] = bmax16(part[q][t], part[q][t + stride]);
    }
    __syncthreads();
  }
  if (t < 4) {
    uint4* r = reinterpret_cast<uint4*>(regs + col) + t;
    uint4 old = *r;
    uint4 nw = bmax16(old, part[t][0]);
    if (nw.x != old.x || nw.y != old.y || nw.z != old.z || nw.w != old.w) {
      *r = nw;
      atomicMax(flag, epoch);
      atomicOr(card, 1ull << 63);
    }
  }
}

void hll_add_launch(rsk_ctx* c, const DevKeys& k, uint8_t* d_regs_sketch, uint64_t* d_card, uint32_t* d_flag,
                    uint32_t epoch, bool created) {
  if (k.n == 0) return;
  constexpr uint64_t T = RSK_ADD_THREADS;
  const uint64_t max_blocks = c->slab_count;
  // Enough keys per workgroup to amortise the 64 KiB LDS init + 16 KiB slab;
  // a persistent grid of the 2 workgroups per CU that the 64 KiB file allows.
  uint64_t blocks = (k.n + 4 * T - 1) / (4 * T);
  blocks = std::min<uint64_t>(blocks, std::min<uint64_t>(2ull * c->num_cus, max_blocks));
  if (blocks == 0) blocks = 1;
  uint64_t per_block = (k.n + blocks - 1) / blocks;
  if (k.offsets == nullptr && k.fixed_len == 16 && (reinterpret_cast<uintptr_t>(k.data) & 15) == 0) {
    // Round the slice up to whole tiles so every lane's loads stay coalesced.
    constexpr uint64_t T16 = 256;
    const uint64_t tile = T16 * RSK_ADD_UNROLL;
    blocks = std::min<uint64_t>((k.n + tile - 1) / tile, std::min<uint64_t>(2ull * c->num_cus, max_blocks));
    per_block = (k.n + blocks - 1) / blocks;
    per_block = (per_block + tile - 1) / tile * tile;
    blocks = (k.n + per_block - 1) / per_block;
    ProfScope ps(c, "hll_add16");
    hipLaunchKernelGGL((hll_add16_kernel<RSK_ADD_UNROLL, T16>), dim3((uint32_t)blocks), dim3(T16), 0, c->stream,
                       reinterpret_cast<const uint4*>(k.data), k.n, per_block, c->d_slab);
    RSK_CHECK_LAUNCH("hll_add16");
  } else if (k.offsets == nullptr) {
    ProfScope ps(c, "hll_add_fixed");
    hipLaunchKernelGGL(hll_add_bytes_kernel<false>, dim3((uint32_t)blocks), dim3(T), 0, c->stream, k.data, nullptr,
                       k.fixed_len, k.n, per_block, c->d_slab);
    RSK_CHECK_LAUNCH("hll_add_fixed");
  } else {
    var_grid(c, k.n, &blocks, &per_block);
    ProfScope ps(c, "hll_add_var");
    hipLaunchKernelGGL(hll_add_var_staged_kernel<1>, dim3((uint32_t)blocks), dim3(VAR_TILE), 0, c->stream, k.data,
                       k.offsets, k.n, per_block, c->d_slab);
    RSK_CHECK_LAUNCH("hll_add_var");
  }
  ProfScope ps(c, "hll_reduce");
  hipLaunchKernelGGL(hll_reduce_kernel, dim3(HLL_REGS / 64), dim3(256), 0, c->stream, c->d_slab, (uint32_t)blocks,
                     d_regs_sketch, d_flag, epoch, reinterpret_cast<unsigned long long*>(d_card), created ? 1 : 0);
  RSK_CHECK_LAUNCH("hll_reduce");
}

// dst = max(dst, src) for one sketch; flag if dst grew (PFMERGE from raw).
__global__ __launch_bounds__(256) void hll_max_into_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                           uint32_t* __restrict__ flag) {
  const int j = blockIdx.x * 256 + threadIdx.x;  // uint4 index, 1024 total
  uint4* d = reinterpret_cast<uint4*>(dst) + j;
  uint4 a = *d, b = reinterpret_cast<const uint4*>(src)[j];
  uint4 m = bmax16(a, b);
  if (m.x != a.x || m.y != a.y || m.z != a.z || m.w != a.w) {
    *d = m;
    if (flag) atomicOr(flag, 1u);
  }
}

void hll_max_into_launch(rsk_ctx* c, uint8_t* d_dst, const uint8_t* d_src, uint32_t* d_flag) {
  ProfScope ps(c, "hll_max_into");
  hipLaunchKernelGGL(hll_max_into_kernel, dim3(HLL_REGS / 16 / 256), dim3(256), 0, c->stream, d_dst, d_src, d_flag);
  RSK_CHECK_LAUNCH("hll_max_into");
}

// --------------------------------------------------------- grouped PFADD
// Pair i -> sketch groups[i]; byte-max on the register's u32 word by CAS.
__global__ __launch_bounds__(256) void hll_add_grouped16_kernel(const uint4* __restrict__ keys,
                                                                const uint32_t* __restrict__ groups, uint64_t n,
                                                                uint8_t* __restrict__ regs, uint64_t G) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = ld_nt16(&keys[i]);
    uint32_t g = __builtin_nontemporal_load(&groups[i]);
    if (g >= G) continue;
    uint64_t h = murmur64a_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z);
    uint32_t idx = hll_index(h), rank = hll_rank(h);
    uint32_t* word = reinterpret_cast<uint32_t*>(regs + (uint64_t)g * HLL_REGS + (idx & ~3u));
    const uint32_t sh = (idx & 3u) * 8;
    uint32_t old = *word;
    while (((old >> sh) & 0xFF) < rank) {
      uint32_t nw = (old & ~(0xFFu << sh)) | (rank << sh);
      uint32_t prev = atomicCAS(word, old, nw);
      if (prev == old) break;
      old = prev;
    }
  }
}

__global__ __launch_bounds__(256) void hll_add_grouped_bytes_kernel(const uint8_t* __restrict__ data,
                                                                    const uint64_t* __restrict__ offsets,
                                                                    uint32_t fixed_len,
                                                                    const uint32_t* __restrict__ groups, uint64_t n,
                                                                    uint8_t* __restrict__ regs, uint64_t G) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t g = groups[i];
    if (g >= G) continue;
    uint64_t s = offsets ? offsets[i] : i * fixed_len;
    uint64_t len = offsets ? offsets[i + 1] - s : fixed_len;
    uint64_t h = murmur64a(data + s, len);
    uint32_t idx = hll_index(h), rank = hll_rank(h);
    uint32_t* word = reinterpret_cast<uint32_t*>(regs + (uint64_t)g * HLL_REGS + (idx & ~3u));
    const uint32_t sh = (idx & 3u) * 8;
    uint32_t old = *word;
    while (((old >> sh) & 0xFF) < rank) {
      uint32_t nw = (old & ~(0xFFu << sh)) | (rank << sh);
      uint32_t prev = atomicCAS(word, old, nw);
      if (prev == old) break;
      old = prev;
    }
  }
}

void hll_add_grouped_launch(rsk_ctx* c, const DevKeys& k, const uint32_t* d_groups, uint8_t* d_regs, uint64_t G,
                            bool pool_zero, bool write_all, PCount pc) {
  if (k.n == 0) return;
  if (hll_add_grouped_partitioned(c, k, d_groups, d_regs, G, pool_zero, write_all, pc)) return;  // large batches: per-sketch LDS updates
  uint64_t blocks = (k.n + 255) / 256;
  uint64_t cap = (uint64_t)c->num_cus * 16;
  if (blocks > cap) blocks = cap;
  if (k.offsets == nullptr && k.fixed_len == 16 && (reinterpret_cast<uintptr_t>(k.data) & 15) == 0) {
    ProfScope ps(c, "hll_add_grouped16");
    hipLaunchKernelGGL(hll_add_grouped16_kernel, dim3((uint32_t)blocks), dim3(256), 0, c->stream,
                       reinterpret_cast<const uint4*>(k.data), d_groups, k.n, d_regs, G);
    RSK_CHECK_LAUNCH("hll_add_grouped16");
  } else {
    ProfScope ps(c, "hll_add_grouped");
    hipLaunchKernelGGL(hll_add_grouped_bytes_kernel, dim3((uint32_t)blocks), dim3(256), 0, c->stream, k.data,
                       k.offsets, k.fixed_len, d_groups, k.n, d_regs, G);
    RSK_CHECK_LAUNCH("hll_add_grouped");
  }
}

// ---------------------------------------------------------------- PFCOUNT
// One sketch's 16 KiB as 16 uint4 per lane of a wave.
RSK_DEV SumD wave_sum(const uint4 (&v)[16]) {
  SumD s{0.0, 0, 0};
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    acc_word(s, v[q].x);
    acc_word(s, v[q].y);
    acc_word(s, v[q].z);
    acc_word(s, v[q].w);
  }
  return wave_reduce(s);
}

RSK_DEV double dense_order_sum(const uint8_t* r, int* ezp) {
  double E = 0;
  int ez = 0;
  for (int g = 0; g < HLL_REGS / 16; ++g) {
    const uint8_t* q = r + 16 * g;
    for (int t = 0; t < 16; ++t) ez += q[t] == 0;
    E += (pe(q[0]) + pe(q[1])) + (pe(q[2]) + pe(q[3])) + (pe(q[4]) + pe(q[5])) + (pe(q[6]) + pe(q[7])) +
         (pe(q[8]) + pe(q[9])) + (pe(q[10]) + pe(q[11])) + (pe(q[12]) + pe(q[13])) + (pe(q[14]) + pe(q[15]));
  }
  *ezp = ez;
  return E;
}

// PFCOUNT, one wave per sketch: the 16 KiB are 16 uint4 loads per lane, all
// in flight at once; no LDS and no barrier.
__global__ __launch_bounds__(256) void hll_count_kernel(const uint8_t* __restrict__ regs, uint64_t* __restrict__ card,
                                                        const uint64_t* __restrict__ ids, SmallIds small, uint64_t n,
                                                        const double* __restrict__ lc, uint64_t* __restrict__ out,
                                                        PCount pc) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  for (uint64_t b = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; b < n; b += nwaves) {
    const uint64_t id = ids ? ids[b] : (small.n ? small.v[b] : b);
    const uint64_t cached = card[id];
    if ((cached >> 63) == 0) {  // HLL_VALID_CACHE
      if (lane == 0) out[b] = cached;
      continue;
    }
    if (pc.pcount && pc.pepoch[id] == pc.epoch) {  // estimated by the grouped add from these registers
      if (lane == 0) {
        const uint64_t est = pc.pcount[id];
        out[b] = est;
        card[id] = est;
      }
      continue;
    }
    const uint8_t* r = regs + id * HLL_REGS;
    const uint4* r4 = reinterpret_cast<const uint4*>(r) + lane;
    uint4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = r4[64 * q];
    const SumD s = wave_sum(v);
    if (lane == 0) {
      int ez = (int)s.ez;
      const double E = exact_total(s) ? s.t : dense_order_sum(r, &ez);
      const uint64_t est = hll_estimate(E, ez, lc);
      out[b] = est;
      card[id] = est;  // cache refreshed, valid
    }
  }
}

void hll_count_launch(rsk_ctx* c, const uint8_t* d_regs, uint64_t* d_card, const uint64_t* d_ids,
                      const SmallIds& small, uint64_t n, uint64_t* d_out, PCount pc) {
  if (n == 0) return;
  uint64_t grid = (n + 3) / 4;  // 4 waves (sketches) per workgroup
  if (grid > (1u << 20)) grid = 1u << 20;
  ProfScope ps(c, "hll_count");
  hipLaunchKernelGGL(hll_count_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, d_regs, d_card, d_ids, small, n,
                     c->d_lc, d_out, pc);
  RSK_CHECK_LAUNCH("hll_count");
}

RSK_DEV double raw_order_sum(const uint8_t* const* members, uint32_t arity, int* ezp) {
  double E = 0;
  int ez = 0;
  for (int j = 0; j < HLL_REGS / 8; ++j) {
    uint8_t b[8];
    uint64_t word = 0;
    for (int t = 0; t < 8; ++t) {
      uint8_t m = 0;
      for (uint32_t a = 0; a < arity; ++a) {
        uint8_t x = members[a][8 * j + t];
        m = x > m ? x : m;
      }
      b[t] = m;
      word |= (uint64_t)m << (8 * t);
    }
    if (word == 0) {
      ez += 8;
    } else {
      for (int t = 0; t < 8; ++t) {
        if (b[t]) E += pe(b[t]);
        else ez++;
      }
    }
  }
  E += ez;
  *ezp = ez;
  return E;
}

// Multi-key PFCOUNT: union of `arity` sketches into HLL_RAW, raw-order sum.
__global__ __launch_bounds__(256) void hll_union_count_kernel(const uint8_t* const* __restrict__ member_ptrs,
                                                              uint32_t arity, uint64_t n,
                                                              const double* __restrict__ lc,
                                                              uint64_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  for (uint64_t b = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; b < n; b += nwaves) {  // one wave per union
    const uint8_t* const* mem = member_ptrs + b * arity;
    uint4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = make_uint4(0, 0, 0, 0);
    for (uint32_t a = 0; a < arity; ++a) {
      if (mem[a] == nullptr) continue;
      const uint4* p = reinterpret_cast<const uint4*>(mem[a]) + lane;
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = bmax16(v[q], p[64 * q]);
    }
    const SumD s = wave_sum(v);
    if (lane == 0) {
      int ez = (int)s.ez;
      double E = s.t;
      if (!exact_total(s)) {
        // Absent members contribute zeros: compact the pointer list.
        const uint8_t* live[64];
        uint32_t na = 0;
        for (uint32_t a = 0; a < arity && na < 64; ++a)
          if (mem[a]) live[na++] = mem[a];
        E = raw_order_sum(live, na, &ez);
      }
      out[b] = hll_estimate(E, ez, lc);
    }
  }
}

void hll_union_count_launch(rsk_ctx* c, const uint8_t* const* d_member_ptrs, uint32_t arity, uint64_t n,
                            uint64_t* d_out) {
  if (n == 0) return;
  uint64_t grid = (n + 3) / 4;  // 4 waves (unions) per workgroup
  if (grid > (1u << 20)) grid = 1u << 20;
  ProfScope ps(c, "hll_union_count");
  hipLaunchKernelGGL(hll_union_count_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, d_member_ptrs, arity, n,
                     c->d_lc, d_out);
  RSK_CHECK_LAUNCH("hll_union_count");
}

// PFMERGE: dst[i] = max(dst[i], srcs[i][0..k)); null src = absent key.
__global__ __launch_bounds__(256) void hll_merge_kernel(uint8_t* const* __restrict__ dst_ptrs,
                                                        const uint8_t* const* __restrict__ src_ptrs, uint32_t k,
                                                        uint64_t n) {
  for (uint64_t b = blockIdx.x; b < n; b += gridDim.x) {
    uint4* d = reinterpret_cast<uint4*>(dst_ptrs[b]);
    const uint8_t* const* srcs = src_ptrs + b * k;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = threadIdx.x + 256 * q;
      uint4 v = d[j];
      for (uint32_t a = 0; a < k; ++a)
        if (srcs[a]) v = bmax16(v, reinterpret_cast<const uint4*>(srcs[a])[j]);
      d[j] = v;
    }
  }
}

void hll_merge_launch(rsk_ctx* c, uint8_t* const* d_dst_ptrs, const uint8_t* const* d_src_ptrs, uint32_t srcs_per_dst,
                      uint64_t n) {
  if (n == 0) return;
  uint64_t grid = n < (1u << 20) ? n : (1u << 20);
  ProfScope ps(c, "hll_merge");
  hipLaunchKernelGGL(hll_merge_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, d_dst_ptrs, d_src_ptrs,
                     srcs_per_dst, n);
  RSK_CHECK_LAUNCH("hll_merge");
}

// ------------------------------------------- PFADD one element at a time
// Element i replies 1 iff rank_i > max(reg0[idx_i], ranks of earlier
// elements with the same index).  Elements are radix-sorted by register
// index (stable, so input order survives inside a register); the "earlier
// ranks" term is then an exclusive segmented max-scan over the sorted ranks
// (rocprim scan-by-key), so a register hit by many elements (a skewed or
// duplicate-heavy batch) costs no more than one spread over all registers.
__global__ void hll_each_hash_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                                     uint32_t fixed_len, uint64_t n, uint32_t* __restrict__ key_idx,
                                     uint32_t* __restrict__ seq, uint8_t* __restrict__ rank) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t s = offsets ? offsets[i] : i * fixed_len;
    uint64_t len = offsets ? offsets[i + 1] - s : fixed_len;
    uint64_t h = murmur64a(data + s, len);
    key_idx[i] = hll_index(h);
    seq[i] = (uint32_t)i;
    rank[i] = (uint8_t)hll_rank(h);
  }
}

__global__ void hll_each_gather_kernel(const uint32_t* __restrict__ sorted_seq, const uint8_t* __restrict__ rank,
                                       uint64_t n, uint32_t* __restrict__ sorted_rank) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x)
    sorted_rank[p] = rank[sorted_seq[p]];
}

// Replies in input order; the last element of each run leaves the register's
// new value in next_reg (regs itself is only read here).
__global__ void hll_each_reply_kernel(const uint32_t* __restrict__ sorted_idx, const uint32_t* __restrict__ sorted_seq,
                                      const uint32_t* __restrict__ sorted_rank, const uint32_t* __restrict__ prefix,
                                      uint64_t n, const uint8_t* __restrict__ regs, uint8_t* __restrict__ out,
                                      uint32_t* __restrict__ next_reg) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = sorted_idx[p];
    const uint32_t base = regs[r];
    const uint32_t pre = prefix[p] > base ? prefix[p] : base;
    const uint32_t c = sorted_rank[p];
    out[sorted_seq[p]] = c > pre;
    if (p + 1 == n || sorted_idx[p + 1] != r) next_reg[r] = c > pre ? c : pre;
  }
}

__global__ void hll_each_store_kernel(const uint32_t* __restrict__ next_reg, uint8_t* __restrict__ regs) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < HLL_REGS && next_reg[r] != 0xFFFFFFFFu) regs[r] = (uint8_t)next_reg[r];
}

void hll_add_each_launch(rsk_ctx* c, const DevKeys& k, const uint8_t* d_regs_sketch, uint8_t* d_out) {
  // d_regs_sketch is updated in place (const only for signature symmetry).
  uint8_t* regs = const_cast<uint8_t*>(d_regs_sketch);
  const uint64_t n = k.n;
  if (n == 0) return;
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, HLL_P, c->stream);
  (void)hipcub::DeviceScan::ExclusiveScanByKey(nullptr, scan_bytes, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                                               (uint32_t*)nullptr, hipcub::Max(), 0u, (uint32_t)n,
                                               hipcub::Equality(), c->stream);
  size_t tmp_bytes = std::max(sort_bytes, scan_bytes);
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  uint64_t need = 4 * al(n * 4) + al(n) + al(HLL_REGS * 4) + al(tmp_bytes);
  uint8_t* w = c->work(need);
  uint32_t* idx_in = reinterpret_cast<uint32_t*>(w);
  uint32_t* idx_out = reinterpret_cast<uint32_t*>(w + al(n * 4));
  uint32_t* seq_in = reinterpret_cast<uint32_t*>(w + 2 * al(n * 4));
  uint32_t* seq_out = reinterpret_cast<uint32_t*>(w + 3 * al(n * 4));
  uint8_t* rank = w + 4 * al(n * 4);
  uint32_t* next_reg = reinterpret_cast<uint32_t*>(w + 4 * al(n * 4) + al(n));
  void* tmp = w + 4 * al(n * 4) + al(n) + al(HLL_REGS * 4);
  // After the sort the unsorted key/seq arrays are free: sorted ranks and
  // the scan's output reuse them.
  uint32_t* sorted_rank = idx_in;
  uint32_t* prefix = seq_in;
  uint64_t grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  ProfScope ps(c, "hll_add_each");
  hipLaunchKernelGGL(hll_each_hash_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, k.data, k.offsets,
                     k.fixed_len, n, idx_in, seq_in, rank);
  RSK_CHECK_LAUNCH("hll_each_hash");
  RSK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, sort_bytes, idx_in, idx_out, seq_in, seq_out, (int)n, 0, HLL_P,
                                             c->stream));
  hipLaunchKernelGGL(hll_each_gather_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, seq_out, rank, n,
                     sorted_rank);
  RSK_CHECK_LAUNCH("hll_each_gather");
  RSK_HIP(hipcub::DeviceScan::ExclusiveScanByKey(tmp, scan_bytes, (const uint32_t*)idx_out,
                                                 (const uint32_t*)sorted_rank, prefix, hipcub::Max(), 0u, (uint32_t)n,
                                                 hipcub::Equality(), c->stream));
  RSK_HIP(hipMemsetAsync(next_reg, 0xFF, HLL_REGS * 4, c->stream));
  hipLaunchKernelGGL(hll_each_reply_kernel, dim3((uint32_t)grid), dim3(256), 0, c->stream, idx_out, seq_out,
                     sorted_rank, prefix, n, regs, d_out, next_reg);
  RSK_CHECK_LAUNCH("hll_each_reply");
  hipLaunchKernelGGL(hll_each_store_kernel, dim3(HLL_REGS / 256), dim3(256), 0, c->stream, next_reg, regs);
  RSK_CHECK_LAUNCH("hll_each_store");
}

}  // namespace rsk
