// rsk_bloom_pg.hip -- Bloom insert for large batches by paged partition (gfx950).
//
// RedissonBloomFilter.add (src/main/java/org/redisson/RedissonBloomFilter.java:80-114)
// sets k bits per element (k SETBITs, :94-98) at idx_t = (h_t & Long.MAX_VALUE)
// % size (:116-131).  Setting bits is an OR, so the probes may be applied in
// any order; they are routed to 64 KiB slices of the filter (2^19 bits), each
// slice then ORed in LDS and written back once.  Two routing passes, each of
// which APPENDS bin runs to 4 KiB pages (1024 probes) of its own private
// region, so that every later read is of whole pages:
//
//   pg1   : workgroup w hashes its contiguous key range once (XXH64 +
//           farmhash; <= 16 probes per lane in registers), a tile at a time:
//           ranks the probes by coarse bin (idx >> (19 + f2), <= 256 bins) with
//           one LDS atomic each, places them bin-sorted in an LDS image, and
//           appends each bin's run to that bin's current page (new pages come
//           from the workgroup's own page counter: no global atomics, no
//           histogram pass).  At the end it lists its pages by bin.
//   size  : per (coarse bin c, group g of pg1 workgroups): probes in, and the
//           pg2 region offsets (prefix sums).
//   pg2   : workgroup (c, g) streams the pages of bin c of its pg1
//           workgroups (16 chunks of 64 probes per page), ranks by fine bin
//           (the 2^f2 slices of c, probes 19 bits), and appends runs to pages
//           of its own region the same way, then lists them by slice.
//   apply : workgroup per slice: 64 KiB of filter in LDS, every page of that
//           slice (from the NG pg2 workgroups of its coarse bin) ORed in with
//           ds_or, 16 loads in flight per page; the slice written back once.
// Filters of <= 256 slices skip pg2 (apply reads the pg1 pages).
//
// HBM per key at k probes: 16 B of key + 4k (pg1) + 4k + 4k (pg2) + 4k (apply),
// plus 2 x the filter per chunk and < 0.2 % of page bookkeeping.
#include <cstdlib>
#include <cstring>

#include "rsk_internal.h"

namespace rsk {

namespace {

constexpr int SL_LOG = 19;                            // bits per slice
constexpr uint32_t SL_WORDS = 1u << (SL_LOG - 5);     // 16384 u32 = 64 KiB of LDS
constexpr uint32_t SL_MAX = 32768;                    // slices (2^34 bits) handled here
constexpr uint32_t PG = 1024;                         // probes per page (4 KiB)
constexpr int R2 = 14;                                // pg2 probe slots of 64 per lane and tile
constexpr int TA = 1024;                              // apply workgroup
constexpr uint32_t INVALID = 0xFFFFFFFFu;             // no probe (payloads are < 2^26)
constexpr uint64_t DEFAULT_PROBE_CHUNK = 1ull << 33;  // probes per chunk (2 x 32 GiB of pages)

RSK_DEV uint32_t rdl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
RSK_DEV uint32_t sgpr(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

RSK_DEV uint32_t wave_scan_incl(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  return x;
}

// Page cursors of one workgroup's bins (LDS).  A bin's current page is cur[b]
// holding fill[b] probes; fill == PG means no room (also before the first page).
// Per tile: run start in the image (lstart), where the run's first `room`
// probes go (dst0, a probe index in the region), the first of its new pages (blk).
template <int NB>
struct PageState {
  uint32_t cur[NB], fill[NB], npages[NB];
  uint32_t lstart[NB + 1], room[NB], blk[NB];
  uint32_t dst0[NB];
  uint32_t pages_used;
};

template <int NB>
RSK_DEV void page_state_init(PageState<NB>& S, uint32_t nb) {
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
    S.cur[b] = 0;
    S.fill[b] = PG;
    S.npages[b] = 0;
  }
  if (threadIdx.x == 0) S.pages_used = 0;
}

// Wave 0: a tile's bin counts (hist, zeroed here) -> run starts, and pages for
// every run: the part that fits the bin's current page, the rest in a block of
// consecutive new pages from the workgroup's counter; log[page] = bin.
template <int NB>
RSK_DEV void wave0_plan(uint32_t* hist, PageState<NB>& S, uint32_t nb, uint8_t* __restrict__ log) {
  constexpr int PER = NB / 64;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t cnt[PER], need[PER], sum = 0, nsum = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t b = lane * PER + i;
    cnt[i] = b < nb ? hist[b] : 0;
    if (b < nb) hist[b] = 0;
    const uint32_t room = b < nb ? PG - S.fill[b] : 0;
    need[i] = cnt[i] > room ? (cnt[i] - room + PG - 1) / PG : 0;
    sum += cnt[i];
    nsum += need[i];
  }
  const uint32_t incl = wave_scan_incl(sum, lane), nincl = wave_scan_incl(nsum, lane);
  uint32_t run = incl - sum, pg = S.pages_used + nincl - nsum;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t b = lane * PER + i;
    if (b < nb) {
      const uint32_t fill = S.fill[b], room = PG - fill;
      S.lstart[b] = run;
      S.room[b] = cnt[i] < room ? cnt[i] : room;
      S.dst0[b] = S.cur[b] * PG + fill;
      S.blk[b] = pg;
      for (uint32_t j = 0; j < need[i]; ++j) log[pg + j] = (uint8_t)b;
      if (need[i]) {
        S.cur[b] = pg + need[i] - 1;
        S.fill[b] = cnt[i] - room - (need[i] - 1) * PG;
        S.npages[b] += need[i];
      } else {
        S.fill[b] = fill + cnt[i];
      }
    }
    run += cnt[i];
    pg += need[i];
  }
  const uint32_t tot = rdl(incl, 63), ntot = rdl(nincl, 63);
  if (lane == 0) {
    S.lstart[nb] = tot;
    S.pages_used += ntot;
  }
}

// Write-out of a bin-sorted tile image: wave w copies the runs of bins
// w, w + NW, ... (rank r < room -> the current page, the rest -> the block).
template <int NB>
RSK_DEV void write_runs(const uint32_t* img, const PageState<NB>& S, uint32_t nb, uint32_t nw,
                        uint32_t* __restrict__ region, uint32_t mask) {
  const uint32_t lane = threadIdx.x & 63, w = sgpr(threadIdx.x >> 6);
  for (uint32_t b = w; b < nb; b += nw) {
    const uint32_t st = S.lstart[b], len = S.lstart[b + 1] - st, room = S.room[b];
    const uint64_t d0 = S.dst0[b], d1 = (uint64_t)S.blk[b] * PG;
    for (uint32_t r = lane; r < len; r += 64) {
      const uint64_t d = r < room ? d0 + r : d1 + (r - room);
      region[d] = img[st + r] & mask;
    }
  }
}

// End of a workgroup: its pages listed by bin (order inside a bin is free),
// list_off[b] = start of bin b's list (n_pages at [nb]), last[b] = its last
// page's id and fill (pages before it are full).
template <int NB>
RSK_DEV void list_pages(PageState<NB>& S, uint32_t nb, const uint8_t* __restrict__ log,
                        uint32_t* __restrict__ list, uint32_t* __restrict__ list_off,
                        uint32_t* __restrict__ last_page, uint32_t* __restrict__ last_fill, uint32_t* cursor) {
  __syncthreads();
  if (threadIdx.x < 64) {
    constexpr int PER = NB / 64;
    const uint32_t lane = threadIdx.x;
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t b = lane * PER + i;
      v[i] = b < nb ? S.npages[b] : 0;
      sum += v[i];
    }
    const uint32_t incl = wave_scan_incl(sum, lane);
    uint32_t run = incl - sum;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t b = lane * PER + i;
      if (b < nb) {
        cursor[b] = run;
        list_off[b] = run;
        last_page[b] = S.cur[b];
        last_fill[b] = v[i] ? S.fill[b] : 0;
      }
      run += v[i];
    }
    if (lane == 63) list_off[nb] = incl;
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < S.pages_used; p += blockDim.x) list[atomicAdd(&cursor[log[p]], 1u)] = p;
}

RSK_DEV void key_words(const uint4& v, uint64_t* w0, uint64_t* w1) {
  *w0 = ((uint64_t)v.y << 32) | v.x;
  *w1 = ((uint64_t)v.w << 32) | v.z;
}

// The pages of one bin (or slice) held by up to MAXS "sources" (producer
// workgroups) as one concatenated list: per source the page-count prefix, the
// bin's list start, its last page / fill, and the source's region base (pages;
// its lists start there too).  Loaded by wave 0 into LDS.
constexpr uint32_t MAXS = 512;
struct SrcTable {
  uint32_t pre[MAXS + 1], start[MAXS], lastp[MAXS], lastf[MAXS];
  uint64_t base[MAXS];
};

// src(i, &row, &base): source i's row of the per-bin arrays and region base.
template <class F>
RSK_DEV void wave0_sources(SrcTable& T, uint32_t ns, uint32_t bin, uint32_t nbp1, const uint32_t* __restrict__ list_off,
                           const uint32_t* __restrict__ last_page, const uint32_t* __restrict__ last_fill, F&& src) {
  constexpr int PER = MAXS / 64;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t si = lane * PER + i;
    v[i] = 0;
    if (si < ns) {
      uint64_t row, base;
      src(si, &row, &base);
      const uint32_t* lo = list_off + row * nbp1 + bin;
      const uint32_t a = lo[0];
      v[i] = lo[1] - a;
      T.start[si] = a;
      T.lastp[si] = last_page[row * nbp1 + bin];
      T.lastf[si] = last_fill[row * nbp1 + bin];
      T.base[si] = base;
    }
    sum += v[i];
  }
  const uint32_t incl = wave_scan_incl(sum, lane);
  uint32_t run = incl - sum;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t si = lane * PER + i;
    if (si < ns) T.pre[si] = run;
    run += v[i];
  }
  if (lane == 63) T.pre[ns] = incl;
}

// Source of page j of the concatenated list (j < T.pre[ns]): the largest i
// with pre[i] <= j (empty sources share their successor's prefix).
RSK_DEV uint32_t find_source(const SrcTable& T, uint32_t ns, uint32_t j) {
  uint32_t lo = 0, hi = ns;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (T.pre[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// A page of the list: probe address and count.  fetch() issues the list load
// for page j; open() completes it (the load has had the current page's time).
struct PageCursor {
  uint32_t src = 0, pid = 0;
  RSK_DEV void fetch(const SrcTable& T, uint32_t ns, const uint32_t* __restrict__ lists, uint32_t j) {
    src = sgpr(find_source(T, ns, j));
    pid = lists[T.base[src] + T.start[src] + (j - T.pre[src])];
  }
  RSK_DEV void open(const SrcTable& T, uint64_t* addr, uint32_t* cnt) const {
    const uint32_t p = sgpr(pid);
    *cnt = p == T.lastp[src] ? T.lastf[src] : PG;
    *addr = (T.base[src] + p) * (uint64_t)PG;
  }
};

// ------------------------------------------------------------------- pg1
// Workgroup w: tiles [w * tpw, (w+1) * tpw) of KST keys; its pages at
// out + w * cap_pages * PG, page log / lists at [w * cap_pages ...],
// per-bin list offsets / last pages at [w * (nb1 + 1) ...].
template <bool FIXED16, int KMAX, int T1>
__global__ __launch_bounds__(T1) void bloom_pg1_kernel(const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ offsets, uint32_t fixed_len,
                                                       uint64_t n, FastMod63 fm, int k, uint32_t shift1, uint32_t nb1,
                                                       uint64_t tpw, uint64_t cap_pages, uint32_t* __restrict__ out,
                                                       uint8_t* __restrict__ logs, uint32_t* __restrict__ lists,
                                                       uint32_t* __restrict__ list_off,
                                                       uint32_t* __restrict__ last_page,
                                                       uint32_t* __restrict__ last_fill) {
  constexpr int KPL = 16 / KMAX;        // keys per lane
  constexpr uint32_t KST = T1 * KPL;    // keys per tile
  constexpr int NP = KPL * KMAX;        // probe slots per lane (16)
  __shared__ __attribute__((aligned(16))) uint32_t img[2][T1 * NP];
  __shared__ uint32_t hist[256];
  __shared__ PageState<256> S;
  const uint64_t low = (1ull << shift1) - 1;
  const uint64_t w = blockIdx.x;
  const uint64_t nst = (n + KST - 1) / KST;
  const uint64_t st_beg = w * tpw, st_end = st_beg + tpw < nst ? st_beg + tpw : nst;
  uint32_t* region = out + w * cap_pages * PG;
  uint8_t* log = logs + w * cap_pages;
  if (threadIdx.x < 256) hist[threadIdx.x] = 0;
  page_state_init(S, nb1);
  const uint4* keys16 = reinterpret_cast<const uint4*>(data);
  uint4 nxt[KPL];
  auto fetch = [&](uint64_t st) {
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const uint64_t i = st * KST + threadIdx.x + (uint64_t)u * T1;
      nxt[u] = (FIXED16 && st < st_end && i < n) ? ld_nt16(keys16 + i) : make_uint4(0, 0, 0, 0);
    }
  };
  if (FIXED16) fetch(st_beg);
  __syncthreads();
  uint32_t buf = 0;
  for (uint64_t st = st_beg; st < st_end; ++st, buf ^= 1) {
    const uint64_t k0 = st * KST;
    const uint32_t nk = (uint32_t)(n - k0 < KST ? n - k0 : KST);
    uint4 cur[KPL];
#pragma unroll
    for (int u = 0; u < KPL; ++u) cur[u] = nxt[u];
    if (FIXED16) fetch(st + 1);  // the next tile's keys stream in meanwhile
    uint32_t pay[NP], tag[NP];
#pragma unroll
    for (int u = 0; u < KPL; ++u) {
      const uint32_t q = threadIdx.x + u * T1;
      const bool ok = q < nk;
      uint64_t h1 = 0, h2 = 0;
      if (ok) {
        if (FIXED16) {
          uint64_t w0, w1;
          key_words(cur[u], &w0, &w1);
          h1 = xxh64_16(w0, w1);
          h2 = farm_16(w0, w1);
        } else {
          bloom_key_hashes<false>(data, offsets, fixed_len, k0 + q, h1, h2);
        }
      }
      ProbeSeq ps(h1, h2, fm);
#pragma unroll
      for (int t = 0; t < KMAX; ++t) {
        const int s = u * KMAX + t;
        tag[s] = INVALID;
        pay[s] = 0;
        if (ok && t < k) {
          const uint64_t idx = ps.idx;
          const uint32_t bin = (uint32_t)(idx >> shift1);
          pay[s] = (uint32_t)(idx & low);
          tag[s] = (bin << 16) | atomicAdd(&hist[bin], 1u);
          if (t + 1 < k) ps.next(t, fm);
        }
      }
    }
    __syncthreads();  // (A) every rank taken
    if (threadIdx.x < 64) wave0_plan<256>(hist, S, nb1, log);
    __syncthreads();  // (B) run starts and pages planned, hist zeroed
    uint32_t* im = img[buf];  // last read by the write-out two tiles back, before every wave reached (B)
#pragma unroll
    for (int s = 0; s < NP; ++s)
      if (tag[s] != INVALID) im[S.lstart[tag[s] >> 16] + (tag[s] & 0xFFFFu)] = pay[s];
    __syncthreads();  // (C) image complete
    write_runs<256>(im, S, nb1, T1 / 64, region, 0xFFFFFFFFu);
  }
  list_pages<256>(S, nb1, log, lists + w * cap_pages, list_off + w * (nb1 + 1), last_page + w * (nb1 + 1),
                  last_fill + w * (nb1 + 1), hist);
}

// ---------------------------------------------------------------- sizing
// (c, g): probes of coarse bin c in the pages of pg1 workgroups [g*GU, (g+1)*GU)
// -> pages2[cp] = pg2 region capacity (its pages + one spare per fine bin).
__global__ __launch_bounds__(256) void pg_size_kernel(const uint32_t* __restrict__ list_off,
                                                      const uint32_t* __restrict__ last_fill, uint32_t nb1,
                                                      uint32_t G1, uint32_t GU, uint32_t NG, uint32_t nb2,
                                                      uint64_t* __restrict__ pages2) {
  const uint32_t cp = blockIdx.x * 256 + threadIdx.x;
  if (cp >= nb1 * NG) return;
  const uint32_t c = cp / NG, g = cp - c * NG;
  uint64_t probes = 0;
  for (uint32_t w = g * GU; w < (g + 1) * GU && w < G1; ++w) {
    const uint32_t* lo = list_off + (uint64_t)w * (nb1 + 1);
    const uint32_t np = lo[c + 1] - lo[c];
    if (np) probes += (uint64_t)(np - 1) * PG + last_fill[(uint64_t)w * (nb1 + 1) + c];
  }
  pages2[cp] = (probes + PG - 1) / PG + nb2;
}

// One workgroup: exclusive prefix sum over n u64 values in place-out (total at [n]).
__global__ __launch_bounds__(1024) void pg_scan_kernel(const uint64_t* __restrict__ in, uint32_t n,
                                                       uint64_t* __restrict__ out) {
  __shared__ uint64_t part[1024];
  const uint32_t per = (n + 1023) / 1024, b0 = threadIdx.x * per;
  uint64_t a = 0;
  for (uint32_t i = b0; i < b0 + per && i < n; ++i) a += in[i];
  part[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t r = 0;
    for (int i = 0; i < 1024; ++i) {
      const uint64_t x = part[i];
      part[i] = r;
      r += x;
    }
    out[n] = r;
  }
  __syncthreads();
  a = part[threadIdx.x];
  for (uint32_t i = b0; i < b0 + per && i < n; ++i) {
    out[i] = a;
    a += in[i];
  }
}

// ------------------------------------------------------------------- pg2
// Workgroup (c, g): the pages of bin c of pg1 workgroups g*GU .. (g+1)*GU - 1,
// wave v taking pages v, v + NW, ... of that concatenated list (GU <= 256:
// list starts / counts of the GU workgroups prefix-summed in LDS).  A wave's
// R2 slots per tile are consecutive 64-probe chunks of its current page.
template <int T2>
__global__ __launch_bounds__(T2) void bloom_pg2_kernel(const uint32_t* __restrict__ in, uint64_t cap1,
                                                       const uint32_t* __restrict__ lists1,
                                                       const uint32_t* __restrict__ list_off1,
                                                       const uint32_t* __restrict__ last_page1,
                                                       const uint32_t* __restrict__ last_fill1, uint32_t nb1,
                                                       uint32_t G1, uint32_t GU, uint32_t NG, uint32_t nb2,
                                                       const uint64_t* __restrict__ base2,
                                                       uint32_t* __restrict__ out, uint8_t* __restrict__ logs2,
                                                       uint32_t* __restrict__ lists2,
                                                       uint32_t* __restrict__ list_off2,
                                                       uint32_t* __restrict__ last_page2,
                                                       uint32_t* __restrict__ last_fill2) {
  constexpr uint32_t NW = T2 / 64;
  __shared__ __attribute__((aligned(16))) uint32_t img[2][T2 * R2];
  __shared__ uint32_t hist[128];
  __shared__ PageState<128> S;
  __shared__ SrcTable T;
  const uint32_t cp = blockIdx.x, c = cp / NG, g = cp - c * NG;
  const uint32_t lane = threadIdx.x & 63, wv = sgpr(threadIdx.x >> 6);
  const uint32_t w0 = g * GU, nsrc = (w0 + GU < G1 ? GU : (G1 > w0 ? G1 - w0 : 0));
  if (threadIdx.x < 128) hist[threadIdx.x] = 0;
  page_state_init(S, nb2);
  if (threadIdx.x < 64)
    wave0_sources(T, nsrc, c, nb1 + 1, list_off1, last_page1, last_fill1, [&](uint32_t si, uint64_t* row, uint64_t* base) {
      *row = w0 + si;
      *base = (uint64_t)(w0 + si) * cap1;
    });
  __syncthreads();
  const uint32_t npages_in = T.pre[nsrc];
  // wave-uniform cursor: page j (of the concatenated list) at chunk q; the
  // next page's list entry is fetched while this one is read
  uint32_t j = wv, q = 0, pcnt = 0;
  uint64_t paddr = 0;
  PageCursor pc;
  bool have = j < npages_in;
  if (have) {
    pc.fetch(T, nsrc, lists1, j);
    pc.open(T, &paddr, &pcnt);
    if (j + NW < npages_in) pc.fetch(T, nsrc, lists1, j + NW);
  }
  uint32_t* region = out + base2[cp] * PG;
  uint8_t* log = logs2 + base2[cp];
  __syncthreads();
  uint32_t buf = 0;
  for (;;) {
    uint32_t pay[R2], tag[R2];
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      pay[r] = INVALID;
      if (have) {
        const uint32_t o = q * 64 + lane;
        if (o < pcnt) pay[r] = __builtin_nontemporal_load(&in[paddr + o]);
        ++q;
        if (q * 64 >= pcnt) {
          j += NW;
          have = j < npages_in;
          if (have) {
            pc.open(T, &paddr, &pcnt);
            q = 0;
            if (j + NW < npages_in) pc.fetch(T, nsrc, lists1, j + NW);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      tag[r] = INVALID;
      if (pay[r] != INVALID) {
        const uint32_t bin = pay[r] >> SL_LOG;
        tag[r] = (bin << 16) | atomicAdd(&hist[bin], 1u);
      }
    }
    const int more = __syncthreads_or(have ? 1 : 0);  // (A) every rank taken
    if (threadIdx.x < 64) wave0_plan<128>(hist, S, nb2, log);
    __syncthreads();  // (B)
    if (S.lstart[nb2]) {
      uint32_t* im = img[buf];
#pragma unroll
      for (int r = 0; r < R2; ++r)
        if (tag[r] != INVALID) im[S.lstart[tag[r] >> 16] + (tag[r] & 0xFFFFu)] = pay[r];
      __syncthreads();  // (C) image complete
      write_runs<128>(im, S, nb2, NW, region, (1u << SL_LOG) - 1);
      buf ^= 1;
    }
    if (!more) break;
  }
  list_pages<128>(S, nb2, log, lists2 + base2[cp], list_off2 + (uint64_t)cp * (nb2 + 1),
                  last_page2 + (uint64_t)cp * (nb2 + 1), last_fill2 + (uint64_t)cp * (nb2 + 1), hist);
}

// ----------------------------------------------------------------- apply
// Slice s: its pages held by NG sources.  Two-level (base2 != nullptr): coarse
// bin c = s >> f2, list f = s & (2^f2 - 1) of pg2 workgroups cp = c * NG + g
// (region / lists at base2[cp]).  One level: list s of pg1 workgroups g (region
// / lists at g * cap).  Wave v takes pages v, v + NW, ...: a page's 16 chunks
// are loaded at once, then ORed in with ds_or; the next page's list entry is
// fetched meanwhile.
template <int UA>
__global__ __launch_bounds__(TA) void bloom_pg_apply_kernel(const uint32_t* __restrict__ probes,
                                                            const uint64_t* __restrict__ base2, uint64_t cap,
                                                            const uint32_t* __restrict__ lists,
                                                            const uint32_t* __restrict__ list_off,
                                                            const uint32_t* __restrict__ last_page,
                                                            const uint32_t* __restrict__ last_fill, uint32_t f2,
                                                            uint32_t nb, uint32_t NG, uint32_t nslices,
                                                            uint32_t* __restrict__ bits, uint64_t nwords) {
  __shared__ __attribute__((aligned(16))) uint32_t sl[SL_WORDS];
  __shared__ SrcTable T;
  constexpr uint32_t NW = TA / 64;
  const uint32_t lane = threadIdx.x & 63, wv = sgpr(threadIdx.x >> 6);
  for (uint32_t s = blockIdx.x; s < nslices; s += gridDim.x) {
    const uint64_t w0 = (uint64_t)s * SL_WORDS;
    const uint32_t nw4 = (uint32_t)((nwords - w0 < SL_WORDS ? nwords - w0 : SL_WORDS) / 4);
    uint4* g4 = reinterpret_cast<uint4*>(bits + w0);
    uint4* l4 = reinterpret_cast<uint4*>(sl);
    for (uint32_t qq = threadIdx.x; qq < nw4; qq += TA) l4[qq] = g4[qq];
    const uint32_t c = base2 ? s >> f2 : 0, f = base2 ? s & ((1u << f2) - 1) : s;
    if (threadIdx.x < 64)
      wave0_sources(T, NG, f, nb + 1, list_off, last_page, last_fill, [&](uint32_t g, uint64_t* row, uint64_t* base) {
        *row = (uint64_t)c * NG + g;
        *base = base2 ? base2[*row] : (uint64_t)g * cap;
      });
    __syncthreads();
    const uint32_t npg = T.pre[NG];
    PageCursor pc;
    if (wv < npg) pc.fetch(T, NG, lists, wv);
    for (uint32_t j = wv; j < npg; j += NW) {
      uint64_t addr;
      uint32_t cnt;
      pc.open(T, &addr, &cnt);
      if (j + NW < npg) pc.fetch(T, NG, lists, j + NW);
      const uint32_t* pp = probes + addr;
      for (uint32_t o0 = 0; o0 < cnt; o0 += 64 * UA) {
        uint32_t v[UA];
#pragma unroll
        for (int u = 0; u < UA; ++u) {
          const uint32_t o = o0 + 64 * u + lane;
          v[u] = o < cnt ? __builtin_nontemporal_load(&pp[o]) : INVALID;
        }
#pragma unroll
        for (int u = 0; u < UA; ++u)
          if (v[u] != INVALID) atomicOr(&sl[v[u] >> 5], bloom_bit_mask(v[u]));
      }
    }
    __syncthreads();
    for (uint32_t qq = threadIdx.x; qq < nw4; qq += TA) g4[qq] = l4[qq];
    __syncthreads();
  }
}

uint32_t env_u32(const char* name, uint32_t dflt) {  // tuning knobs
  const char* e = std::getenv(name);
  return (e && *e) ? (uint32_t)std::strtoul(e, nullptr, 10) : dflt;
}

uint32_t nbits(uint64_t v) {  // bits needed to hold v (0 -> 0)
  uint32_t b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}

// Resident workgroups per CU of a kernel (occupancy API; >= 1).
int resident(const void* kernel, int threads) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    per_cu = 1;
  }
  return per_cu;
}

}  // namespace

bool bloom_add_paged(rsk_ctx* c, rsk_bloom* b, const DevKeys& keys) {
  const char* me = std::getenv("RSK_BLOOM_PG");  // unset: auto; "0": never; "1": always (any batch size)
  const int mode = (!me || !*me) ? -1 : (me[0] == '0' ? 0 : 1);
  const uint64_t k = (uint64_t)b->k;
  const uint64_t nslices = ((uint64_t)b->size + (1ull << SL_LOG) - 1) >> SL_LOG;
  if (mode == 0 || k > 16 || nslices > SL_MAX || keys.n == 0) return false;
  if (mode < 0 && keys.n * k < (1ull << 22)) return false;  // small batches: direct atomics
  const bool f16 =
      keys.offsets == nullptr && keys.fixed_len == 16 && (reinterpret_cast<uintptr_t>(keys.data) & 15) == 0;
  const uint32_t kmax = k <= 8 ? 8 : 16;
  const uint32_t t1 = env_u32("RSK_BLOOM_PG_T1", 512) == 1024 ? 1024 : 512;
  const uint32_t t2 = env_u32("RSK_BLOOM_PG_T2", 1024) == 512 ? 512 : 1024;
  const uint32_t ua = env_u32("RSK_BLOOM_PG_UA", 16) == 8 ? 8 : 16;
  const uint64_t kst = (uint64_t)t1 * (16 / kmax);
  const uint32_t sb = nbits(nslices - 1);
  const uint32_t f2 = sb > 8 ? sb - 8 : 0;
  const uint32_t shift1 = SL_LOG + f2;
  const uint32_t nb1 = (uint32_t)(((nslices - 1) >> f2) + 1);
  const uint32_t nb2 = 1u << f2;
  const uint32_t ns = (uint32_t)nslices;
  const uint32_t cus = (uint32_t)c->num_cus;
  // pg1 workgroups: as many as are resident at once (one contiguous key range each)
  const void* k1 = t1 == 1024 ? (const void*)bloom_pg1_kernel<true, 8, 1024> : (const void*)bloom_pg1_kernel<true, 8, 512>;
  const uint32_t G1max = std::min<uint32_t>(MAXS, (uint32_t)resident(k1, (int)t1) * cus);
  uint64_t chunk = std::max<uint64_t>(1, (env_u32("RSK_BLOOM_PG_CHUNK", 0) ? env_u32("RSK_BLOOM_PG_CHUNK", 0)
                                                                            : DEFAULT_PROBE_CHUNK) / k / kst) * kst;
  chunk = std::min<uint64_t>(chunk, keys.n);
  const uint64_t max_nst = (chunk + kst - 1) / kst;
  const uint32_t G1 = (uint32_t)std::min<uint64_t>(G1max, max_nst);
  const uint64_t tpw = (max_nst + G1 - 1) / G1;                     // tiles per pg1 workgroup
  const uint64_t cap1 = (tpw * kst * k + PG - 1) / PG + nb1;        // pages per pg1 region
  // pg2 groups: about 4 workgroups per CU over the nb1 coarse bins, GU <= 256 sources each
  uint32_t NG = f2 ? std::max<uint32_t>(1, (4 * cus + nb1 - 1) / nb1) : G1;
  NG = std::min<uint32_t>(NG, G1);
  const uint32_t GU = (G1 + NG - 1) / NG;
  NG = (G1 + GU - 1) / GU;
  const uint32_t ncp = nb1 * NG;
  const uint64_t pages1 = (uint64_t)G1 * cap1;
  const uint64_t pages2_max = f2 ? pages1 + (uint64_t)ncp * nb2 + ncp : 0;  // >= sum of pg2 capacities
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  const uint64_t per1 = (uint64_t)G1 * (nb1 + 1), per2 = (uint64_t)ncp * (nb2 + 1);
  const uint64_t bytes = al(4 * pages1 * PG) + al(pages1) + al(4 * pages1) + 3 * al(4 * per1) +
                         (f2 ? al(4 * pages2_max * PG) + al(pages2_max) + al(4 * pages2_max) + 3 * al(4 * per2) +
                                   2 * al(8 * (ncp + 1))
                             : 0);
  uint8_t* wk = c->work(bytes);
  uint8_t* q = wk;
  auto take = [&](uint64_t nbytes) {
    uint8_t* r = q;
    q += al(nbytes);
    return r;
  };
  uint32_t* pg1 = reinterpret_cast<uint32_t*>(take(4 * pages1 * PG));
  uint8_t* log1 = take(pages1);
  uint32_t* lists1 = reinterpret_cast<uint32_t*>(take(4 * pages1));
  uint32_t* off1 = reinterpret_cast<uint32_t*>(take(4 * per1));
  uint32_t* lastp1 = reinterpret_cast<uint32_t*>(take(4 * per1));
  uint32_t* lastf1 = reinterpret_cast<uint32_t*>(take(4 * per1));
  uint32_t *pg2 = nullptr, *lists2 = nullptr, *off2 = nullptr, *lastp2 = nullptr, *lastf2 = nullptr;
  uint8_t* log2 = nullptr;
  uint64_t *cap2 = nullptr, *base2 = nullptr;
  if (f2) {
    pg2 = reinterpret_cast<uint32_t*>(take(4 * pages2_max * PG));
    log2 = take(pages2_max);
    lists2 = reinterpret_cast<uint32_t*>(take(4 * pages2_max));
    off2 = reinterpret_cast<uint32_t*>(take(4 * per2));
    lastp2 = reinterpret_cast<uint32_t*>(take(4 * per2));
    lastf2 = reinterpret_cast<uint32_t*>(take(4 * per2));
    cap2 = reinterpret_cast<uint64_t*>(take(8 * (ncp + 1)));
    base2 = reinterpret_cast<uint64_t*>(take(8 * (ncp + 1)));
  }

  for (uint64_t first = 0; first < keys.n; first += chunk) {
    const uint64_t m = std::min<uint64_t>(chunk, keys.n - first);
    const uint64_t nst = (m + kst - 1) / kst;
    const uint32_t g1 = (uint32_t)((nst + tpw - 1) / tpw);  // workgroups with tiles (<= G1)
    DevKeys dk = keys;
    dk.n = m;
    if (keys.offsets) dk.offsets = keys.offsets + first;
    else dk.data = keys.data + first * keys.fixed_len;
    {
      ProfScope ps(c, "bloom_pg1");
#define RSK_PG1(F16, KM, TT)                                                                                   \
  hipLaunchKernelGGL((bloom_pg1_kernel<F16, KM, TT>), dim3(g1), dim3(TT), 0, c->stream, dk.data, dk.offsets, \
                     dk.fixed_len, m, b->fm, b->k, shift1, nb1, tpw, cap1, pg1, log1, lists1, off1, lastp1, lastf1)
      if (t1 == 1024) {
        if (f16 && kmax == 8) RSK_PG1(true, 8, 1024);
        else if (f16) RSK_PG1(true, 16, 1024);
        else if (kmax == 8) RSK_PG1(false, 8, 1024);
        else RSK_PG1(false, 16, 1024);
      } else {
        if (f16 && kmax == 8) RSK_PG1(true, 8, 512);
        else if (f16) RSK_PG1(true, 16, 512);
        else if (kmax == 8) RSK_PG1(false, 8, 512);
        else RSK_PG1(false, 16, 512);
      }
#undef RSK_PG1
      RSK_CHECK_LAUNCH("bloom_pg1");
    }
    const uint32_t ng = f2 ? (g1 + GU - 1) / GU : g1;  // sources per coarse bin this chunk
    if (f2) {
      const uint32_t ncpc = nb1 * ng;
      {
        ProfScope ps(c, "bloom_pg_mid");
        hipLaunchKernelGGL(pg_size_kernel, dim3((ncpc + 255) / 256), dim3(256), 0, c->stream, off1, lastf1, nb1, g1,
                           GU, ng, nb2, cap2);
        RSK_CHECK_LAUNCH("bloom_pg_size");
        hipLaunchKernelGGL(pg_scan_kernel, dim3(1), dim3(1024), 0, c->stream, cap2, ncpc, base2);
        RSK_CHECK_LAUNCH("bloom_pg_scan");
      }
      {
        ProfScope ps(c, "bloom_pg2");
        if (t2 == 512)
          hipLaunchKernelGGL(bloom_pg2_kernel<512>, dim3(ncpc), dim3(512), 0, c->stream, pg1, cap1, lists1, off1,
                             lastp1, lastf1, nb1, g1, GU, ng, nb2, base2, pg2, log2, lists2, off2, lastp2, lastf2);
        else
          hipLaunchKernelGGL(bloom_pg2_kernel<1024>, dim3(ncpc), dim3(1024), 0, c->stream, pg1, cap1, lists1, off1,
                             lastp1, lastf1, nb1, g1, GU, ng, nb2, base2, pg2, log2, lists2, off2, lastp2, lastf2);
        RSK_CHECK_LAUNCH("bloom_pg2");
      }
    }
    {
      ProfScope ps(c, "bloom_pg_apply");
      const int per_cu = resident((const void*)bloom_pg_apply_kernel<16>, TA);
      const uint32_t grid = (uint32_t)std::min<uint64_t>(ns, (uint64_t)per_cu * cus);
#define RSK_APPLY(U)                                                                                             \
  if (f2)                                                                                                        \
    hipLaunchKernelGGL((bloom_pg_apply_kernel<U>), dim3(grid), dim3(TA), 0, c->stream, pg2, base2, (uint64_t)0,  \
                       lists2, off2, lastp2, lastf2, f2, nb2, ng, ns, b->d_bits, b->nwords);                    \
  else                                                                                                           \
    hipLaunchKernelGGL((bloom_pg_apply_kernel<U>), dim3(grid), dim3(TA), 0, c->stream, pg1,                      \
                       (const uint64_t*)nullptr, cap1, lists1, off1, lastp1, lastf1, 0u, nb1, g1, ns, b->d_bits, \
                       b->nwords)
      if (ua == 8) RSK_APPLY(8);
      else RSK_APPLY(16);
#undef RSK_APPLY
      RSK_CHECK_LAUNCH("bloom_pg_apply");
    }
  }
  return true;
}

}  // namespace rsk
