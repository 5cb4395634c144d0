// rsk_comm.hip -- device memory API and the RCCL merge layer.
//
// Multi-GPU layout: one process per GPU, the key stream split
// into contiguous ranges, every GPU builds full sketches, and the only
// exchange is the merge:
//   HLL   : ncclAllReduce(uint8, ncclMax) over the 16 KiB register file
//           (bit-exact: max is associative and commutative) -- latency-bound;
//   pools : the same over [n][16384] (bandwidth-bound, ring over xGMI), or a
//           reduce-scatter that leaves rank r owning a contiguous 1/N of the
//           sketches (the C5 plan: half the traffic of the all-reduce);
//   Bloom : RCCL has no bitwise OR, so all-to-all of 1/N slices and, after a
//           local OR, all-to-all of the merged slices back (grouped
//           ncclSend/ncclRecv straight out of / into the filter).
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "rsk_internal.h"

using rsk::RskError;

namespace {

#define RSK_NCCL(expr)                                                                                   \
  do {                                                                                                   \
    ncclResult_t _r = (expr);                                                                            \
    if (_r != ncclSuccess)                                                                               \
      throw RskError{RSK_ERR_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(_r)};                \
  } while (0)

template <class F>
int guarded(F&& fn) {
  try {
    fn();
    rsk::set_error("");
    return RSK_OK;
  } catch (const RskError& e) {
    rsk::set_error(e.msg);
    return e.code;
  } catch (const std::exception& e) {
    rsk::set_error(e.what());
    return RSK_ERR_DEVICE;
  }
}

void need(bool cond, const char* msg) {
  if (!cond) throw RskError{RSK_ERR_INVALID_ARG, msg};
}

struct Lock {
  std::lock_guard<std::recursive_mutex> g;
  explicit Lock(rsk_ctx* c) : g(c->mu) { RSK_HIP(hipSetDevice(c->device)); }
};

ncclComm_t comm_of(rsk_ctx* c) {
  need(c->comm != nullptr, "no communicator: call rsk_comm_init first");
  return reinterpret_cast<ncclComm_t>(c->comm);
}

// One point-to-point transfer as pieces of at most 1 GiB (a 4 GB self
// send/recv of the routed add's records came back wrong in one piece, 1 GiB
// pieces right; the pieces to one peer are matched in issue order on both
// sides).  Every row / slice / record exchange below goes through it.
constexpr uint64_t P2P_PIECE = 1ull << 30;
void p2p_pieces(const void* buf, uint64_t bytes, int peer, ncclComm_t comm, hipStream_t s, bool send) {
  for (uint64_t o = 0; o < bytes; o += P2P_PIECE) {
    const uint64_t m = std::min(P2P_PIECE, bytes - o);
    const uint8_t* p = static_cast<const uint8_t*>(buf) + o;
    if (send) RSK_NCCL(ncclSend(p, m, ncclUint8, peer, comm, s));
    else RSK_NCCL(ncclRecv(const_cast<uint8_t*>(p), m, ncclUint8, peer, comm, s));
  }
}

__global__ void invalidate_card_kernel(uint64_t* card, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    card[i] |= (1ull << 63);
}

// Row exchange (rsk_hll_fetch_rows): 16 KiB sketch rows between the pool and
// a contiguous staging buffer, one workgroup per row, 16-byte lanes.
constexpr uint32_t ROW_U4 = rsk::HLL_REGS / 16;  // 1024 uint4 per sketch

__global__ __launch_bounds__(256) void gather_rows_kernel(const uint4* __restrict__ pool, const uint64_t* __restrict__ ids,
                                                          uint64_t n, uint4* __restrict__ out) {
  for (uint64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const uint4* src = pool + ids[r] * ROW_U4;
    uint4* dst = out + r * ROW_U4;
    for (uint32_t q = threadIdx.x; q < ROW_U4; q += 256) dst[q] = src[q];
  }
}

__global__ __launch_bounds__(256) void scatter_rows_kernel(uint4* __restrict__ pool, uint64_t* __restrict__ card,
                                                           const uint64_t* __restrict__ ids, uint64_t n,
                                                           const uint4* __restrict__ in) {
  for (uint64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const uint64_t id = ids[r];
    uint4* dst = pool + id * ROW_U4;
    const uint4* src = in + r * ROW_U4;
    for (uint32_t q = threadIdx.x; q < ROW_U4; q += 256) dst[q] = src[q];
    if (threadIdx.x == 0) card[id] |= (1ull << 63);
  }
}

}  // namespace

extern "C" {

int rsk_dev_alloc(rsk_ctx* c, uint64_t bytes, void** out) {
  return guarded([&] {
    need(c && out, "NULL argument");
    Lock l(c);
    *out = nullptr;
    RSK_HIP(hipMalloc(out, bytes ? bytes : 1));
  });
}

int rsk_dev_free(rsk_ctx* c, void* p) {
  return guarded([&] {
    need(c != nullptr, "ctx is NULL");
    Lock l(c);
    if (p) {
      RSK_HIP(hipStreamSynchronize(c->stream));
      RSK_HIP(hipFree(p));
    }
  });
}

int rsk_memcpy(rsk_ctx* c, void* dst, const void* src, uint64_t bytes, uint32_t kind) {
  return guarded([&] {
    need(c && (bytes == 0 || (dst && src)), "NULL argument");
    need(kind <= RSK_D2D, "bad copy kind");
    Lock l(c);
    const hipMemcpyKind k = kind == RSK_H2D ? hipMemcpyHostToDevice
                            : kind == RSK_D2H ? hipMemcpyDeviceToHost
                                              : hipMemcpyDeviceToDevice;
    if (bytes) RSK_HIP(hipMemcpyAsync(dst, src, bytes, k, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_memset(rsk_ctx* c, void* p, int value, uint64_t bytes) {
  return guarded([&] {
    need(c && (p || bytes == 0), "NULL argument");
    Lock l(c);
    if (bytes) RSK_HIP(hipMemsetAsync(p, value, bytes, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_comm_unique_id(uint8_t* id_out) {
  return guarded([&] {
    need(id_out != nullptr, "NULL argument");
    ncclUniqueId id;
    RSK_NCCL(ncclGetUniqueId(&id));
    std::memcpy(id_out, id.internal, RSK_COMM_ID_BYTES);
  });
}

int rsk_comm_init(rsk_ctx* c, int nranks, int rank, const uint8_t* id) {
  return guarded([&] {
    need(c && id, "NULL argument");
    need(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
    Lock l(c);
    if (c->comm) {
      (void)ncclCommDestroy(reinterpret_cast<ncclComm_t>(c->comm));
      c->comm = nullptr;
    }
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, RSK_COMM_ID_BYTES);
    ncclComm_t comm;
    RSK_NCCL(ncclCommInitRank(&comm, nranks, uid, rank));
    c->comm = comm;
    c->nranks = nranks;
    c->rank = rank;
  });
}

// What RCCL itself reports for the context's communicator (not the arguments
// rsk_comm_init was given): a bench line or a test can then show that every
// rank joined.  Without a communicator: 1 rank, rank 0.
int rsk_comm_info(rsk_ctx* c, int* nranks, int* rank) {
  return guarded([&] {
    need(c && nranks && rank, "NULL argument");
    Lock l(c);
    if (!c->comm) {
      *nranks = 1;
      *rank = 0;
      return;
    }
    int n = 0, r = -1;
    RSK_NCCL(ncclCommCount(reinterpret_cast<ncclComm_t>(c->comm), &n));
    RSK_NCCL(ncclCommUserRank(reinterpret_cast<ncclComm_t>(c->comm), &r));
    *nranks = n;
    *rank = r;
  });
}

int rsk_comm_destroy(rsk_ctx* c) {
  return guarded([&] {
    need(c != nullptr, "ctx is NULL");
    Lock l(c);
    if (c->comm) {
      RSK_HIP(hipStreamSynchronize(c->stream));
      RSK_NCCL(ncclCommDestroy(reinterpret_cast<ncclComm_t>(c->comm)));
      c->comm = nullptr;
    }
    c->nranks = 1;
    c->rank = 0;
  });
}

int rsk_hll_allreduce(rsk_hll* h, uint64_t id) {
  return guarded([&] {
    need(h != nullptr, "bad sketch");
    rsk_ctx* c = h->ctx;
    Lock l(c);
    ncclComm_t comm = comm_of(c);
    // A bad id on one rank must not strand the others in the collective: that
    // rank reduces a scratch row and reports the error after it.
    const bool ok = id < h->n;
    uint8_t* regs = ok ? h->d_regs + id * (uint64_t)rsk::HLL_REGS : c->work(rsk::HLL_REGS);
    if (ok) {
      rsk::hll_materialize(h);
      rsk::hll_touch(h);
      rsk::hll_forget_import(h, id);
    } else {
      RSK_HIP(hipMemsetAsync(regs, 0, rsk::HLL_REGS, c->stream));
    }
    {
      rsk::ProfScope ps(c, "hll_allreduce");
      RSK_NCCL(ncclAllReduce(regs, regs, rsk::HLL_REGS, ncclUint8, ncclMax, comm, c->stream));
    }
    RSK_HIP(hipStreamSynchronize(c->stream));
    need(ok, "sketch id out of range");
    hipLaunchKernelGGL(invalidate_card_kernel, dim3(1), dim3(64), 0, c->stream, h->d_card + id, (uint64_t)1);
    RSK_CHECK_LAUNCH("invalidate");
    h->exists[id] = 1;
    h->dense[id] = 1;
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_hll_allreduce_pool(rsk_hll* h) {
  return guarded([&] {
    need(h != nullptr, "bad pool");
    rsk_ctx* c = h->ctx;
    Lock l(c);
    rsk::hll_materialize(h);
    rsk::hll_touch(h);
    rsk::hll_forget_imports(h);
    ncclComm_t comm = comm_of(c);
    {
      rsk::ProfScope ps(c, "hll_allreduce_pool");
      RSK_NCCL(ncclAllReduce(h->d_regs, h->d_regs, h->n * (uint64_t)rsk::HLL_REGS, ncclUint8, ncclMax, comm,
                             c->stream));
    }
    hipLaunchKernelGGL(invalidate_card_kernel, dim3(256), dim3(256), 0, c->stream, h->d_card, h->n);
    RSK_CHECK_LAUNCH("invalidate");
    std::fill(h->exists.begin(), h->exists.end(), 1);
    std::fill(h->dense.begin(), h->dense.end(), 1);
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_hll_reducescatter_pool(rsk_hll* h, uint64_t* first_out, uint64_t* count_out) {
  return guarded([&] {
    need(h && first_out && count_out, "NULL argument");
    rsk_ctx* c = h->ctx;
    Lock l(c);
    rsk::hll_materialize(h);
    rsk::hll_touch(h);
    rsk::hll_forget_imports(h);
    ncclComm_t comm = comm_of(c);
    const uint64_t N = (uint64_t)c->nranks, r = (uint64_t)c->rank, R = rsk::HLL_REGS;
    const uint64_t q = h->n / N, tail = h->n - q * N;
    {
      rsk::ProfScope ps(c, "hll_reducescatter_pool");
      // In place: rank r's slice of the send buffer is its receive buffer.
      if (q) RSK_NCCL(ncclReduceScatter(h->d_regs, h->d_regs + r * q * R, q * R, ncclUint8, ncclMax, comm, c->stream));
      // The last n mod N sketches are reduced on every rank (owned by the last).
      if (tail) RSK_NCCL(ncclAllReduce(h->d_regs + q * N * R, h->d_regs + q * N * R, tail * R, ncclUint8, ncclMax, comm,
                                       c->stream));
    }
    hipLaunchKernelGGL(invalidate_card_kernel, dim3(256), dim3(256), 0, c->stream, h->d_card, h->n);
    RSK_CHECK_LAUNCH("invalidate");
    std::fill(h->exists.begin(), h->exists.end(), 1);
    std::fill(h->dense.begin(), h->dense.end(), 1);
    rsk::plan_owned_range(h->n, N, r, first_out, count_out);
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

// The owner-routed grouped add (C5 across GPUs): pairs hashed
// where they live, 8-byte records shipped to the rank owning their sketch,
// applied there to the owned rows only.  Against building every sketch on
// every rank and reduce-scattering the pool, per rank at N = 8 and the C5
// size (500M pairs, 10^6 sketches): 7/8 x 4 GB of records over xGMI instead
// of 7/8 x 16 GiB of rows, and 2 GiB of rows written instead of 16 GiB.
//
// Skew (VERDICT r05 Weak 6b): with contiguous ownership a Zipf(1.1) stream
// sends 93 % of all pairs to rank 0 at N = 8.  A group with at least
// HEAVY_MIN = 2048 pairs on a rank (16 KiB of records = one row) is folded
// there into a local 16 KiB row (the same record pipeline, onto a scratch pool
// of the heavy groups), and the row travels instead of its records; the owner
// max-merges the rows it receives into its rows after its own apply.  A rank's
// own groups are never pre-combined (no transfer to save; the apply folds
// their records anyway).  Heavy
// groups are found from a sample (hll_heavy_select), which changes only where
// a pair is folded, never the registers (max is order-free).
constexpr uint64_t HEAVY_MIN = 2048;
constexpr uint32_t HEAVY_CAP = 65536;  // heavy rows per rank and call (1 GiB)

__global__ __launch_bounds__(256) void max_rows_kernel(uint4* __restrict__ pool, const uint32_t* __restrict__ ids,
                                                       uint64_t m, const uint4* __restrict__ rows,
                                                       uint32_t* __restrict__ pepoch) {
  // registers are < 64, so a byte max is one SWAR compare: bit 7 of
  // (a | 0x80) - b is set iff a >= b, with no borrow between the bytes
  auto bmax = [](uint32_t a, uint32_t b) {
    const uint32_t ge = ((a | 0x80808080u) - b) & 0x80808080u;
    const uint32_t mk = (ge >> 7) * 0xFFu;
    return (a & mk) | (b & ~mk);
  };
  for (uint64_t r = blockIdx.x; r < m; r += gridDim.x) {
    const uint32_t id = ids[r];
    uint4* dst = pool + (uint64_t)id * ROW_U4;
    const uint4* src = rows + r * ROW_U4;
    for (uint32_t q = threadIdx.x; q < ROW_U4; q += 256) {
      const uint4 a = dst[q], b = src[q];
      dst[q] = make_uint4(bmax(a.x, b.x), bmax(a.y, b.y), bmax(a.z, b.z), bmax(a.w, b.w));
    }
    if (threadIdx.x == 0) pepoch[id] = 0;  // the apply's precomputed PFCOUNT no longer holds
  }
}

int rsk_hll_add_grouped_routed(rsk_hll* h, const rsk_keys* keys, const uint32_t* groups, uint32_t flags,
                               uint64_t* first_out, uint64_t* count_out) {
  return guarded([&] {
    need(h && first_out && count_out, "NULL argument");
    rsk_ctx* c = h->ctx;
    Lock l(c);
    ncclComm_t comm = comm_of(c);
    // TEST ONLY (route route_vranks, 1-rank communicator): plan as rank route_vrank of
    // route_vranks -- its owned sub-range, records for other owners dropped, as if every
    // other rank held no pairs -- so one GPU exercises the sub-range offsets
    const bool virt = c->nranks == 1 && c->tune.route_vranks > 1;
    const uint64_t N = virt ? (uint64_t)c->tune.route_vranks : (uint64_t)c->nranks;
    const uint64_t r = virt ? (uint64_t)c->tune.route_vrank : (uint64_t)c->rank;
    need(r < N, "route_vrank outside route_vranks");
    auto peer = [&](uint64_t j) { return virt ? 0 : (int)j; };  // the communicator rank of plan rank j
    auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
    auto on_gpu = [&](const void* p) {
      hipPointerAttribute_t a{};
      if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
      }
      return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
    };
    // local argument errors are agreed on by every rank before anything moves
    const uint64_t n = keys ? keys->n : 0;
    const bool args_ok =
        keys != nullptr && (flags & ~RSK_FETCH_SELF) == 0 && N <= 64 && h->n <= 0xFFFFFFFFull &&
        (n == 0 || (keys->location == RSK_MEM_DEVICE && keys->offsets == nullptr && keys->fixed_len == 16 &&
                    (reinterpret_cast<uintptr_t>(keys->data) & 15) == 0 && groups != nullptr && on_gpu(keys->data) &&
                    on_gpu(groups)));
    const bool self = (flags & RSK_FETCH_SELF) != 0;  // own records / rows also through RCCL
    const uint64_t G = h->n;
    // heavy-group pre-combine: on where it can move bytes off the links (N > 1, or the
    // self exchange that tests it), for large batches; route_heavy forces it (tests)
    const int hv = c->tune.route_heavy;
    const uint64_t heavy_min = hv > 0 ? (uint64_t)hv : HEAVY_MIN;
    const bool heavy_try = args_ok && hv >= 0 && (N > 1 || self) && n > 0 && G <= (1ull << 28) &&
                           (hv > 0 || n >= (1ull << 22));
    const uint32_t B = rsk::route_blocks(c);
    const uint64_t NO = N + 1;  // owners + the heavy run
    const uint64_t hs_bytes = heavy_try ? rsk::hll_heavy_scratch_bytes(G, HEAVY_CAP) : 0;
    uint8_t* w = c->work(al(8 * 3) + al(4 * NO * B) + al(8 * NO * B) + 2 * al(16 * N) + al(hs_bytes));
    uint64_t* d_meta = reinterpret_cast<uint64_t*>(w);
    uint32_t* d_cnt = reinterpret_cast<uint32_t*>(w + al(24));
    uint64_t* d_off = reinterpret_cast<uint64_t*>(w + al(24) + al(4 * NO * B));
    uint64_t* d_scnt = reinterpret_cast<uint64_t*>(w + al(24) + al(4 * NO * B) + al(8 * NO * B));
    uint64_t* d_rcnt = d_scnt + al(16 * N) / 8;
    uint8_t* d_hscratch = w + al(24) + al(4 * NO * B) + al(8 * NO * B) + 2 * al(16 * N);
    uint64_t* h_meta = reinterpret_cast<uint64_t*>(c->h_small + 8192);
    h_meta[0] = args_ok ? 0 : 1;
    h_meta[1] = h->n;
    h_meta[2] = ~h->n;
    RSK_HIP(hipMemcpyAsync(d_meta, h_meta, 24, hipMemcpyHostToDevice, c->stream));
    RSK_NCCL(ncclAllReduce(d_meta, d_meta, 3, ncclUint64, ncclMax, comm, c->stream));
    RSK_HIP(hipMemcpyAsync(h_meta, d_meta, 24, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    need(args_ok, "rsk_hll_add_grouped_routed: keys must be 16-byte aligned fixed 16-byte keys and groups, both in "
                  "device memory; flags RSK_FETCH_SELF or 0; at most 64 ranks");
    need(h_meta[0] == 0, "rsk_hll_add_grouped_routed: another rank passed an invalid argument");
    need(h_meta[1] == ~h_meta[2], "rsk_hll_add_grouped_routed: pool sizes differ across ranks");
    uint64_t first, count;
    rsk::plan_owned_range(h->n, N, r, &first, &count);
    *first_out = first;
    *count_out = count;
    // 0. heavy groups (sampled counts): their pairs become local rows, not records
    std::vector<uint32_t> heavy_ids;
    uint32_t* d_slot_of = nullptr;
    uint32_t* d_hbits = nullptr;
    uint64_t H = 0;
    if (heavy_try) {
      // ~32 samples at the threshold: a group of a quarter of it (Poisson 8) is almost never
      // taken for heavy (1 group in 10^6 at Poisson 2 with 8 samples was ~1000 at C5 uniform)
      const uint32_t stride = (uint32_t)std::max<uint64_t>(1, heavy_min / 32);
      const uint32_t thr = (uint32_t)std::max<uint64_t>(1, (heavy_min + stride - 1) / stride);
      // own groups stay records unless they too go through RCCL (self exchange)
      const uint64_t skip_lo = self ? 0 : first, skip_hi = self ? 0 : first + count;
      H = rsk::hll_heavy_select(c, groups, n, G, stride, thr, skip_lo, skip_hi, HEAVY_CAP, d_hscratch, &d_slot_of,
                                &d_hbits, &heavy_ids);
      if (!H) d_slot_of = d_hbits = nullptr;
    }
    std::vector<uint64_t> hrows(N, 0), hfirst(N + 1, 0);  // heavy rows per owner, their first slot
    rsk::plan_heavy_rows(G, N, heavy_ids.data(), H, &hrows);
    for (uint64_t o = 0; o < N; ++o) hfirst[o + 1] = hfirst[o] + hrows[o];
    // 1. owner counts per block, their offsets in the send buffer (owner-major, the heavy run last)
    std::vector<uint32_t> cnt(NO * B, 0);
    std::vector<uint64_t> off(NO * B);
    // per peer j: [2j] records for j, [2j + 1] heavy rows for j; received into [2N + 2j], [2N + 2j + 1]
    std::vector<uint64_t> scnt(4 * N, 0);
    if (n) {
      rsk::hll_route_count_launch(c, groups, n, G, (uint32_t)N, d_slot_of, d_hbits, d_cnt);
      RSK_HIP(hipMemcpyAsync(cnt.data(), d_cnt, 4 * NO * B, hipMemcpyDeviceToHost, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
    }
    std::vector<uint64_t> sfirst(NO + 1, 0);  // each owner's run in the send buffer
    uint64_t at = 0;
    for (uint64_t o = 0; o < NO; ++o) {
      sfirst[o] = at;
      for (uint64_t b = 0; b < B; ++b) {
        off[o * B + b] = at;
        at += cnt[o * B + b];
      }
    }
    sfirst[NO] = at;
    const uint64_t n_heavy = sfirst[NO] - sfirst[N];  // pairs folded into local rows
    for (uint64_t j = 0; j < N; ++j) {
      scnt[2 * j] = sfirst[j + 1] - sfirst[j];
      scnt[2 * j + 1] = hrows[j];
    }
    // 2. record and row counts both ways
    RSK_HIP(hipMemcpyAsync(d_scnt, scnt.data(), 16 * N, hipMemcpyHostToDevice, c->stream));
    {
      rsk::ProfScope ps(c, "hll_route_counts");
      RSK_NCCL(ncclGroupStart());
      for (uint64_t j = 0; j < N; ++j) {
        if ((j == r && !self) || (virt && j != r)) continue;
        RSK_NCCL(ncclSend(d_scnt + 2 * j, 2, ncclUint64, peer(j), comm, c->stream));
        RSK_NCCL(ncclRecv(d_rcnt + 2 * j, 2, ncclUint64, peer(j), comm, c->stream));
      }
      RSK_NCCL(ncclGroupEnd());
    }
    RSK_HIP(hipMemcpyAsync(scnt.data() + 2 * N, d_rcnt, 16 * N, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    auto rrec = [&](uint64_t j) -> uint64_t& { return scnt[2 * N + 2 * j]; };
    auto rrow = [&](uint64_t j) -> uint64_t& { return scnt[2 * N + 2 * j + 1]; };
    for (uint64_t j = 0; j < N; ++j)
      if (virt && j != r) rrec(j) = rrow(j) = 0;
    if (!self) {  // my own run and rows stay here (used in place)
      rrec(r) = scnt[2 * r];
      rrow(r) = 0;
    }
    uint64_t n_in = 0, rows_in = 0;
    std::vector<uint64_t> rofs(N + 1, 0), rrofs(N + 1, 0);  // each peer's records / rows in the receive buffers
    for (uint64_t j = 0; j < N; ++j) {
      rofs[j + 1] = rofs[j] + rrec(j);
      rrofs[j + 1] = rrofs[j] + rrow(j);
    }
    n_in = rofs[N];
    rows_in = rrofs[N];
    // 3. buffers: records received (+ heavy row ids received), the send side (records +
    // heavy ids), the heavy rows (local + received).  An allocation may fail on one rank
    // only: every rank learns of it (one more MAX all-reduce) before anything moves.
    const uint64_t R = rsk::HLL_REGS;
    uint2* d_recv = nullptr;
    uint32_t* d_rids = nullptr;
    uint2* d_send = nullptr;
    uint32_t* d_hids = nullptr;
    uint8_t* d_lrows = nullptr;
    uint8_t* d_rrows = nullptr;
    int alloc_code = RSK_OK;
    std::string alloc_msg;
    try {
      uint8_t* x = c->xbuf(al(8 * std::max<uint64_t>(n_in, 1)) + al(4 * rows_in));
      d_recv = reinterpret_cast<uint2*>(x);
      d_rids = reinterpret_cast<uint32_t*>(x + al(8 * std::max<uint64_t>(n_in, 1)));
      uint8_t* sb = c->sbuf(al(8 * std::max<uint64_t>(n, 1)) + al(4 * H));
      d_send = reinterpret_cast<uint2*>(sb);
      d_hids = reinterpret_cast<uint32_t*>(sb + al(8 * std::max<uint64_t>(n, 1)));
      if (H + rows_in) {
        d_lrows = c->hrows((H + rows_in) * R);
        d_rrows = d_lrows + H * R;
      }
    } catch (const RskError& e) {
      alloc_code = e.code;
      alloc_msg = e.msg;
    }
    h_meta[0] = alloc_code == RSK_OK ? 0 : 1;
    RSK_HIP(hipMemcpyAsync(d_meta, h_meta, 8, hipMemcpyHostToDevice, c->stream));
    RSK_NCCL(ncclAllReduce(d_meta, d_meta, 1, ncclUint64, ncclMax, comm, c->stream));
    RSK_HIP(hipMemcpyAsync(h_meta, d_meta, 8, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    if (alloc_code != RSK_OK) throw RskError{alloc_code, "rsk_hll_add_grouped_routed: exchange buffers: " + alloc_msg};
    if (h_meta[0] != 0)
      throw RskError{RSK_ERR_OUT_OF_MEMORY, "rsk_hll_add_grouped_routed: another rank could not allocate its exchange "
                                            "buffers"};
    // 4. the records (light pairs to their owners' runs, heavy pairs to the last run)
    if (n) {
      RSK_HIP(hipMemcpyAsync(d_off, off.data(), 8 * NO * B, hipMemcpyHostToDevice, c->stream));
      rsk::hll_route_scatter_launch(c, reinterpret_cast<const uint8_t*>(keys->data), groups, n, G, (uint32_t)N,
                                    d_slot_of, d_hbits, d_off, d_send);
    }
    // 5. heavy pairs folded into local rows (the record pipeline onto a pool of the H heavy
    // groups; it reuses the context's work buffer, which holds nothing live from here on)
    if (H) {
      RSK_HIP(hipMemcpyAsync(d_hids, heavy_ids.data(), 4 * H, hipMemcpyHostToDevice, c->stream));
      rsk::ProfScope ps(c, "hll_route_heavy_rows");
      rsk::hll_add_grouped_recs_launch(c, d_send + sfirst[N], n_heavy, d_lrows, H, true, true,
                                       rsk::PCount{nullptr, nullptr, 0});
    }
    // 6. exchange: per peer its record run, then its heavy row ids and rows (matched in
    // issue order on both sides), every transfer in pieces of <= 1 GiB
    {
      rsk::ProfScope ps(c, "hll_route_exchange");
      RSK_NCCL(ncclGroupStart());
      for (uint64_t j = 0; j < N; ++j) {
        if ((j == r && !self) || (virt && j != r)) continue;
        p2p_pieces(d_send + sfirst[j], scnt[2 * j] * 8, peer(j), comm, c->stream, true);
        p2p_pieces(d_recv + rofs[j], rrec(j) * 8, peer(j), comm, c->stream, false);
        p2p_pieces(d_hids + hfirst[j], hrows[j] * 4, peer(j), comm, c->stream, true);
        p2p_pieces(d_rids + rrofs[j], rrow(j) * 4, peer(j), comm, c->stream, false);
        p2p_pieces(d_lrows + hfirst[j] * R, hrows[j] * R, peer(j), comm, c->stream, true);
        p2p_pieces(d_rrows + rrofs[j] * R, rrow(j) * R, peer(j), comm, c->stream, false);
      }
      RSK_NCCL(ncclGroupEnd());
    }
    if (!self && scnt[2 * r])
      RSK_HIP(hipMemcpyAsync(d_recv + rofs[r], d_send + sfirst[r], scnt[2 * r] * 8, hipMemcpyDeviceToDevice,
                             c->stream));
    // 7. the owned rows [first, first + count): a pending lazy clear of the whole pool is
    // completed on them by the add (every owned row written) and stays pending on every
    // other row (hll_pend_outside: they read as cleared and are zeroed before any other
    // access); owned rows a partial clear left pending are zeroed first
    rsk::hll_forget_imports(h);
    const bool write_all = h->pending_clear;
    if (!write_all) rsk::hll_materialize_range(h, first, count);
    const bool pool_zero = h->zero;
    rsk::hll_touch(h);
    h->pending_clear = false;
    if (write_all && count < h->n) rsk::hll_pend_outside(h, first, count);
    rsk::hll_add_grouped_recs_launch(c, d_recv, n_in, h->d_regs + first * R, count, pool_zero, write_all,
                                     rsk::PCount{h->d_pcount + first, h->d_pepoch + first, h->pc_epoch});
    // 8. heavy rows into the owned rows, one launch per source (ids distinct within one)
    {
      rsk::ProfScope ps(c, "hll_route_rows_merge");
      for (uint64_t j = 0; j < N; ++j) {
        const bool local = j == r && !self;
        const uint64_t m = local ? hrows[r] : rrow(j);
        if (!m) continue;
        const uint32_t* ids = local ? d_hids + hfirst[r] : d_rids + rrofs[j];
        const uint8_t* rows = local ? d_lrows + hfirst[r] * R : d_rrows + rrofs[j] * R;
        hipLaunchKernelGGL(max_rows_kernel, dim3((uint32_t)std::min<uint64_t>(m, 1u << 16)), dim3(256), 0, c->stream,
                           reinterpret_cast<uint4*>(h->d_regs), ids, m, reinterpret_cast<const uint4*>(rows),
                           h->d_pepoch);
        RSK_CHECK_LAUNCH("max_rows");
      }
    }
    if (count) {
      hipLaunchKernelGGL(invalidate_card_kernel, dim3(256), dim3(256), 0, c->stream, h->d_card + first, count);
      RSK_CHECK_LAUNCH("invalidate");
    }
    std::fill(h->exists.begin() + first, h->exists.begin() + first + count, 1);
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_hll_fetch_rows_flags(rsk_hll* h, const uint64_t* ids, uint64_t n, uint32_t flags) {
  return guarded([&] {
    need(h != nullptr, "NULL handle");  // no communicator to agree through without one
    rsk_ctx* c = h->ctx;
    Lock l(c);
    ncclComm_t comm = comm_of(c);
    const uint64_t N = (uint64_t)c->nranks, r = (uint64_t)c->rank, R = rsk::HLL_REGS;
    {  // peers ask only for owned rows (the shared plan); fetched rows are overwritten whole
      uint64_t f0, fc;
      rsk::plan_owned_range(h->n, N, r, &f0, &fc);
      rsk::hll_materialize_range(h, f0, fc);
    }
    rsk::hll_touch(h);
    rsk::hll_forget_imports(h);
    auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
    // Local argument errors (NULL ids, unknown flags, an id outside the pool)
    // are not thrown here: they go into the agreed "bad" word below, so no
    // other rank is left waiting in a collective.
    const bool args_ok = (ids != nullptr || n == 0) && (flags & ~RSK_FETCH_SELF) == 0;
    // Plan (rsk_plan.hip): distinct requested ids ascending = grouped by owner.
    std::vector<uint64_t> want, cnt_out;
    const bool ok_local = args_ok && rsk::plan_fetch(h->n, N, r, ids, n, flags, &want, &cnt_out);
    // Every rank agrees on argument errors (and on the pool size, which fixes
    // every rank's owner map) before any exchange: one MAX all-reduce of
    // {bad, n, ~n}; max(~n) = ~min(n).
    uint64_t* d_meta = reinterpret_cast<uint64_t*>(c->work(al(8 * 3) + al(16 * N)));
    uint64_t* d_cnt = d_meta + al(8 * 3) / 8;
    uint64_t* h_meta = reinterpret_cast<uint64_t*>(c->h_small + 8192);
    h_meta[0] = ok_local ? 0 : 1;
    h_meta[1] = h->n;
    h_meta[2] = ~h->n;
    RSK_HIP(hipMemcpyAsync(d_meta, h_meta, 24, hipMemcpyHostToDevice, c->stream));
    {
      rsk::ProfScope ps(c, "hll_fetch_agree");
      RSK_NCCL(ncclAllReduce(d_meta, d_meta, 3, ncclUint64, ncclMax, comm, c->stream));
    }
    RSK_HIP(hipMemcpyAsync(h_meta, d_meta, 24, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    need(args_ok, "rsk_hll_fetch_rows: ids is NULL or unknown flags");
    need(ok_local, "sketch id out of range");
    need(h_meta[0] == 0, "rsk_hll_fetch_rows: another rank passed an invalid argument");
    need(h_meta[1] == ~h_meta[2], "rsk_hll_fetch_rows: pool sizes differ across ranks");
    // Counts: one u64 each way per peer ([0, N): rows asked of rank j; [N, 2N): rows rank j asks of us).
    std::vector<uint64_t> cnt(2 * N, 0);
    std::copy(cnt_out.begin(), cnt_out.end(), cnt.begin());
    RSK_HIP(hipMemcpyAsync(d_cnt, cnt.data(), 8 * N, hipMemcpyHostToDevice, c->stream));
    {
      rsk::ProfScope ps(c, "hll_fetch_counts");
      RSK_NCCL(ncclGroupStart());
      for (uint64_t j = 0; j < N; ++j) {
        RSK_NCCL(ncclSend(d_cnt + j, 1, ncclUint64, (int)j, comm, c->stream));
        RSK_NCCL(ncclRecv(d_cnt + N + j, 1, ncclUint64, (int)j, comm, c->stream));
      }
      RSK_NCCL(ncclGroupEnd());
    }
    RSK_HIP(hipMemcpyAsync(cnt.data() + N, d_cnt + N, 8 * N, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    // With equal pools and the shared plan a peer only asks for rows this rank
    // owns, so every incoming count is bounded by the owned range.
    uint64_t n_in = 0;
    for (uint64_t j = 0; j < N; ++j) n_in += cnt[N + j];
    const uint64_t n_out = want.size();
    if (n_in == 0 && n_out == 0) return;  // agreed by every peer through the counts
    // work: [want ids | incoming ids | rows we send | rows we receive]
    uint8_t* w = c->work(al(8 * n_out) + al(8 * n_in) + (n_in + n_out) * R);
    uint64_t* d_want = reinterpret_cast<uint64_t*>(w);
    uint64_t* d_in = reinterpret_cast<uint64_t*>(w + al(8 * n_out));
    uint8_t* rows_send = w + al(8 * n_out) + al(8 * n_in);
    uint8_t* rows_recv = rows_send + n_in * R;
    if (n_out) RSK_HIP(hipMemcpyAsync(d_want, want.data(), 8 * n_out, hipMemcpyHostToDevice, c->stream));
    rsk::ProfScope ps(c, "hll_fetch_rows");
    RSK_NCCL(ncclGroupStart());  // the ids each owner must ship
    for (uint64_t j = 0, so = 0, ro = 0; j < N; so += cnt[j], ro += cnt[N + j], ++j) {
      p2p_pieces(d_want + so, cnt[j] * 8, (int)j, comm, c->stream, true);
      p2p_pieces(d_in + ro, cnt[N + j] * 8, (int)j, comm, c->stream, false);
    }
    RSK_NCCL(ncclGroupEnd());
    if (n_in) {
      hipLaunchKernelGGL(gather_rows_kernel, dim3((uint32_t)std::min<uint64_t>(n_in, 1u << 16)), dim3(256), 0,
                         c->stream, reinterpret_cast<const uint4*>(h->d_regs), d_in, n_in,
                         reinterpret_cast<uint4*>(rows_send));
      RSK_CHECK_LAUNCH("gather_rows");
    }
    RSK_NCCL(ncclGroupStart());  // the rows, in request order
    for (uint64_t j = 0, so = 0, ro = 0; j < N; so += cnt[N + j], ro += cnt[j], ++j) {
      p2p_pieces(rows_send + so * R, cnt[N + j] * R, (int)j, comm, c->stream, true);
      p2p_pieces(rows_recv + ro * R, cnt[j] * R, (int)j, comm, c->stream, false);
    }
    RSK_NCCL(ncclGroupEnd());
    if (n_out) {
      hipLaunchKernelGGL(scatter_rows_kernel, dim3((uint32_t)std::min<uint64_t>(n_out, 1u << 16)), dim3(256), 0,
                         c->stream, reinterpret_cast<uint4*>(h->d_regs), h->d_card, d_want, n_out,
                         reinterpret_cast<const uint4*>(rows_recv));
      RSK_CHECK_LAUNCH("scatter_rows");
      for (uint64_t id : want) h->exists[id] = h->dense[id] = 1;
      rsk::hll_unpend(h, want.data(), want.size());  // written whole: no longer pending clear
    }
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_hll_fetch_rows(rsk_hll* h, const uint64_t* ids, uint64_t n) { return rsk_hll_fetch_rows_flags(h, ids, n, 0); }

int rsk_bloom_allreduce_or(rsk_bloom* b) { return rsk_bloom_allreduce_or_flags(b, 0); }

int rsk_bloom_allreduce_or_flags(rsk_bloom* b, uint32_t flags) {
  return guarded([&] {
    need((flags & ~RSK_FETCH_SELF) == 0, "unknown flags");
    need(b != nullptr, "bad filter");
    rsk_ctx* c = b->ctx;
    Lock l(c);
    ncclComm_t comm = comm_of(c);
    ++b->wgen;
    const uint64_t N = (uint64_t)c->nranks, me = (uint64_t)c->rank;
    // Rank j owns words [j*S, j*S + sz(j)) of the filter: S is a multiple of 4
    // (16-byte vector OR) with N*S >= nwords, so the last slices may be short
    // or empty.  Slices travel straight out of and back into the filter (no
    // staging copies); both phases are grouped point-to-point transfers, one
    // per peer, which on a fully connected xGMI node use every link at once.
    // At N = 1 the rank owns the whole filter and nothing moves.
    const uint64_t S = rsk::plan_bloom_slice_words(b->nwords, N);
    auto sz = [&](uint64_t j) {
      const uint64_t lo = std::min(j * S, b->nwords);
      return std::min(lo + S, b->nwords) - lo;
    };
    const uint64_t mine = sz(me), row = (mine + 3) & ~3ull;  // recv rows 16-byte aligned
    // Peers: every other rank; with RSK_FETCH_SELF also this rank itself (its
    // slice makes the round trip through RCCL, so the exchange runs on one GPU).
    std::vector<uint64_t> peers;
    for (uint64_t j = 0; j < N; ++j)
      if (j != me || (flags & RSK_FETCH_SELF)) peers.push_back(j);
    if (!peers.empty() && b->nwords > 0) {
      uint32_t* recv = reinterpret_cast<uint32_t*>(c->work(peers.size() * row * 4 + 256));
      {  // phase 1: every peer's copy of my slice
        rsk::ProfScope ps(c, "bloom_alltoall");
        RSK_NCCL(ncclGroupStart());
        for (size_t r = 0; r < peers.size(); ++r) {
          const uint64_t j = peers[r];
          p2p_pieces(b->d_bits + j * S, sz(j) * 4, (int)j, comm, c->stream, true);
          p2p_pieces(recv + r * row, mine * 4, (int)j, comm, c->stream, false);
        }
        RSK_NCCL(ncclGroupEnd());
      }
      if (mine) rsk::or_rows_into_launch(c, b->d_bits + me * S, recv, (uint32_t)peers.size(), mine, row);
      {  // phase 2: my merged slice to every peer, theirs into my filter
        rsk::ProfScope ps(c, "bloom_allgather");
        RSK_NCCL(ncclGroupStart());
        for (uint64_t j : peers) {
          // my own slice coming back (self exchange) lands in the consumed recv rows
          uint32_t* into = j == me ? recv : b->d_bits + j * S;
          p2p_pieces(b->d_bits + me * S, mine * 4, (int)j, comm, c->stream, true);
          p2p_pieces(into, sz(j) * 4, (int)j, comm, c->stream, false);
        }
        RSK_NCCL(ncclGroupEnd());
      }
    }
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

}  // extern "C"
