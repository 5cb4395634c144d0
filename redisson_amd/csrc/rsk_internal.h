// rsk_internal.h -- host-side internals shared by the librsketch translation
// units (context, handles, error plumbing, kernel launchers).
#pragma once
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <string>
#include <vector>

#include "../../include/rsketch.h"
#include "rsk_device.h"

namespace rsk {

void set_error(const std::string& msg);

struct RskError {
  int code;
  std::string msg;
};

#define RSK_HIP(expr)                                                                           \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess)                                                                       \
      throw ::rsk::RskError{(_e == hipErrorOutOfMemory) ? RSK_ERR_OUT_OF_MEMORY : RSK_ERR_DEVICE, \
                            std::string(#expr) + ": " + hipGetErrorString(_e)};                 \
  } while (0)

#define RSK_CHECK_LAUNCH(name)                                                              \
  do {                                                                                      \
    hipError_t _e = hipGetLastError();                                                      \
    if (_e != hipSuccess)                                                                   \
      throw ::rsk::RskError{RSK_ERR_DEVICE, std::string("launch ") + (name) + ": " + hipGetErrorString(_e)}; \
  } while (0)

// Route overrides of one context.  The library reads no environment
// variables: a context starts with every route automatic (the zero defaults
// below) and only the test and bench support library changes them
// (librsketch_diag.so: rsk_diag_set_route), so behaviour never depends on the
// process that embeds the library.  Every route is bit-exact; they differ in
// speed and scratch only (DESIGN.md 3 lists which batches take which).
struct Tuning {
  int bloom_stream = 0;      // slice-routed insert (st1/apply, sa1/sa2/apply): 0 auto (>= 2^22 probes), 1 any size, -1 never
  int bloom_part = 0;        // exact-offset insert (rsk_bloom_part.hip): 0 auto, 1 any size, -1 never
  uint64_t bloom_chunk = 0;  // probes per chunk of the slice-routed insert (0: 2^33)
  int sa_dbg = 0;            // TIMING ONLY: the insert's sa1 stores each tile contiguously and the insert stops there
  int sa_v = 0;              // the insert's sa2h tile: uint4 per lane, 0 (= 3), 6 or 8
  int sa_hash = 0;           // TIMING ONLY: sa1 without the hashes (1) or hashes and mods (2); wrong filters
  int sa_full = 0;           // -1: sa1 / rp1 without their full-super-tile path (A/B)
  int gpart_dbg = 0;         // TIMING ONLY (C5 rows not written): bit 0 fine-bin rounds stored contiguously, bit 1 no count pass
  int sa_kc = 0;             // the insert's sa1 for k = 7 with k as a constant: 0 yes, -1 no
  int sa_tiny = 0;           // sub-regions of 32 probes: forces the overflow fallbacks
  uint32_t sa_parts = 0;     // sa2 / rp2 parts per coarse bin (0: 4 x CUs / bins)
  int reply = 0;             // add() replies: 0 auto, 1 group-tag pipeline at any size, -1 the sort path
  uint64_t reply_chunk = 0;  // probes per chunk of the group-tag pipeline (0: 2^33)
  int reply_u = 0;           // rp_treply gather chains per lane: 0 (= 2), 1, 2 or 4
  int reply_v = 0;           // rp2 tile: uint4 per lane, 0 (= 8), 3 or 6
  int reply_s = 0;           // rp_tapply: wave steps whose loads are in flight together, 0 (= 2), 1 or 4
  int reply_dbg = 0;         // timing-only rp_tapply forms (bit 0: no folds, bit 1: no T stores); wrong results
  int reply_bal = 0;         // rp_tapply: 0 an equal slice of the bucket's tiles per wave, -1 strided by 1024 (A/B)
  int gpart = 0;             // partitioned grouped PFADD: 0 auto, 1 any size, -1 never
  int gpart_poison = 0;      // timing-free check: fill the fine-bin output with 0xFF first (a hole then shows)
  int io_trace = 0;          // batched export / import: host phase times to stderr
  int io_piece = 0;          // batched export's copy-out pieces, MiB (0: 16)
  int io_drain = 0;          // batched export: 1 = each chunk's copy-out drained before the next chunk (A/B)
  int copy_nt = 0;           // staged host copies: 0 streaming stores, -1 memcpy (A/B)
  int io_pin = 0;            // batched export / import: a pageable buffer >= 256 MiB pinned for the call (0), never (-1)
  int io_engine = 0;         // batched export / import (and large Bloom GET / SET) copies: 0 the fastest SDMA engine
                             // per direction (measured once per context), -1 HIP's copies (A/B), k > 0 engine k - 1
  int gpart_rt = 0;          // hll_gpart2t's round: 0 8192 records, 1 16384 (A/B)
  int gapply_st = 0;         // hll_gapply's row stores: 0 nontemporal, 1 plain (A/B), 2 none (TIMING ONLY)
  int gpart_tm = 1;          // its first pass tile-major (hll_gpart1t, no count pass): 1 yes, 0 no
  int gpart_tile = 0;        // its tile-major first pass: 0 8192-record tiles (2 x 256 lanes per CU), 1 16384 (512 lanes)
  int route_vranks = 0;      // TEST ONLY, 1-rank communicator: the routed grouped add plans as rank route_vrank of
  int route_vrank = 0;       // route_vranks (its owned sub-range; records of other owners dropped)
  int route_heavy = 0;       // routed add's heavy-group pre-combine: 0 auto (>= 2048 pairs, N > 1 or self exchange,
                             // >= 2^22 pairs), -1 never, > 0 on at any size with that many pairs per heavy group
};

// An asynchronous call (rsk_*_async): its host inputs are copied into the
// op's own pinned buffer (so the caller may reuse them at once), its result
// is read back into pinned memory (large ones on the transfer stream), and a
// host function enqueued behind it (hipLaunchHostFunc) files the op for the
// context's completion thread, which computes the reply and invokes the
// caller's callback.  Ops and their buffers are recycled.
struct AsyncOp {
  rsk_ctx* c = nullptr;
  rsk_done_fn cb = nullptr;
  void* user = nullptr;
  int kind = 0;             // how op_complete derives the callback's value
  uint32_t epoch = 0;       // hll add: the call's epoch (reply = flag == epoch || created)
  bool created = false;
  uint64_t value = 0;       // preset value (kinds without a device result)
  uint8_t* h_buf = nullptr; // pinned: staged keys / pointer arrays, then per-key outputs
  uint64_t h_bytes = 0;
  uint8_t* d_buf = nullptr; // device twin
  uint64_t d_bytes = 0;
  uint64_t* h_res = nullptr;  // 64 B pinned result words
  uint8_t* h_out = nullptr;   // per-key outputs read back (inside h_buf)
  uint8_t* user_out = nullptr;
  uint64_t n_out = 0;
  // copy-stream ordering: ev_in (inputs staged on c->xin, the context stream
  // waits for it), ev_out (the context stream's work done, c->xout waits for
  // it before the read-back); on_xfer: completes on c->xout
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  bool on_xfer = false;
  uint64_t seq = 0;         // submission number: callbacks run in this order
  bool failed = false;      // failed by the completion watchdog (its host function may still fire)
};

struct ProfEntry {
  double ms = 0;
  uint64_t launches = 0;
};

// Kernel-time accounting: start/stop events around each launch on the
// context stream, folded into per-kernel totals when read.
struct Profiler {
  bool on = false;
  std::vector<hipEvent_t> free_events;
  struct Pending {
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::map<std::string, ProfEntry> totals;
};

}  // namespace rsk

constexpr int RSK_ADD_THREADS = 512;     // HLL add workgroup (8 waves)
constexpr int RSK_ADD_UNROLL = 4;        // 16-byte keys in flight per lane
constexpr int RSK_MAX_SLABS = 4096;      // partial register files per launch

struct rsk_ctx {
  int device = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  std::recursive_mutex mu;
  // host -> device staging for RSK_MEM_HOST key batches
  uint8_t* d_stage = nullptr;
  uint64_t stage_bytes = 0;
  unsigned stage_threads = 8;
  // double-buffered pinned host stages (filled by host threads while the
  // previous chunk's DMA runs), their device twins and "DMA done" events;
  // pin_off: pinned allocation failed, copy from the pageable source
  uint8_t* h_pin[2] = {nullptr, nullptr};
  uint8_t* d_pin[2] = {nullptr, nullptr};
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
  hipEvent_t ring_ev[8] = {};  // d2h_staged_on: up to 8 pieces of the two stages in flight
  bool pin_off = false;
  // per-workgroup partial register files [slabs][16384] u8
  uint8_t* d_slab = nullptr;
  uint32_t slab_count = 0;
  // small scratch: flags / counters / ids (device) and pinned host mirror
  uint8_t* d_small = nullptr;
  uint8_t* h_small = nullptr;
  uint8_t* h_io = nullptr;  // pinned per-chunk ids / lengths / offsets of the batched export (lazy)
  uint64_t small_bytes = 0;
  // grow-on-demand device scratch for batched calls (released by rsk_trim)
  uint8_t* d_work = nullptr;
  uint64_t work_bytes = 0;
  // grow-on-demand device output scratch, distinct from d_work
  uint8_t* d_out = nullptr;
  uint64_t out_bytes = 0;
  // grow-on-demand pinned host scratch: per-op arrays of batched calls
  // (countWith / mergeWith sketch pointers) built in place and copied with
  // one asynchronous DMA (the call waits for it before returning)
  uint8_t* h_batch = nullptr;
  uint64_t h_batch_bytes = 0;
  // m*log(m/ez) for ez = 0..16384, computed with the host libm (Redis's log)
  double* d_lc = nullptr;
  rsk::Profiler prof;
  // RCCL communicator (multi-GPU merge layer), null when single-GPU
  void* comm = nullptr;
  int nranks = 1;
  int rank = 0;
  // call number written by kernels that report "something changed" (no reset)
  uint32_t epoch = 0;
  rsk::Tuning tune;
  // add()-with-replies counters (rsk_diag_reply_stats): groups whose pending
  // probes were resolved in LDS, chunks answered by the sort-path fallback
  uint64_t rp_pending_groups = 0, rp_fallbacks = 0;
  // asynchronous calls: op pool (a completion returns its op under async_mu)
  std::mutex async_mu;
  std::vector<rsk::AsyncOp*> async_free;
  std::vector<rsk::AsyncOp*> async_all;
  // asynchronous calls' host->device input copies (xin) and device->host
  // read-backs (xout) run on two more streams, ordered against the context
  // stream by events, so they overlap the kernels of earlier calls instead of
  // queueing between them (and inputs never wait behind a read-back)
  hipStream_t xin = nullptr, xout = nullptr;
  // completions: a stream's host function only files its op here (the
  // runtime runs host functions in stream order, so a slow one -- an 8 MB
  // reply copy, a callback waiting for a lock -- would stall the work behind
  // it); done_thr runs them in submission order (ops reach it from two
  // streams, so out of order at times)
  std::thread done_thr;
  std::mutex done_mu;
  std::condition_variable done_cv;
  std::map<uint64_t, rsk::AsyncOp*> done_arrived;  // by seq
  std::map<uint64_t, rsk::AsyncOp*> done_pending;  // submitted, not delivered (by seq)
  uint64_t done_submitted = 0, done_delivered = 0;
  bool done_stop = false;
  // A device error was seen on one of the context's streams while calls were
  // outstanding: their callbacks got RSK_ERR_DEVICE and every later call on
  // the context fails with it (its streams cannot be trusted any more).
  std::atomic<bool> dead{false};

  // grow-on-demand device scratch for collectives' receive buffers (the
  // routed grouped add), distinct from d_work, which the add itself uses
  uint8_t* d_xbuf = nullptr;
  uint64_t xbuf_bytes = 0;
  // the routed grouped add's send side (records, heavy ids) and its heavy
  // rows (built locally and received), grow-on-demand like d_xbuf
  uint8_t* d_sbuf = nullptr;
  uint64_t sbuf_bytes = 0;
  uint8_t* d_hrows = nullptr;
  uint64_t hrows_bytes = 0;
  // large PFCOUNT batches: the list of sketches the cache / precomputed estimate does not answer
  uint8_t* d_cslow = nullptr;
  uint64_t cslow_bytes = 0;

  uint8_t* work(uint64_t bytes);
  uint8_t* pinned(uint64_t bytes);
  // host ranges the caller registered (rsk_host_register) or the export pinned for a call:
  // [base, base + bytes), and the address the device's copy engines use for base (0: unknown)
  struct HostReg {
    uintptr_t base;
    uint64_t bytes;
    uintptr_t dptr;
  };
  std::vector<HostReg> host_regs;
  const HostReg* host_reg(const void* p, uint64_t bytes) const {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (const auto& r : host_regs)
      if (a >= r.base && a + bytes <= r.base + r.bytes) return &r;
    return nullptr;
  }
  bool host_registered(const void* p, uint64_t bytes) const { return host_reg(p, bytes) != nullptr; }
  // The batched export's device->host copies (and the batched import's host->device ones) go
  // to one SDMA engine per direction, the fastest of those measured once per context (round 6:
  // the engine the runtime picks moved 26-30 GB/s on some boxes, 57 on others and on the engines
  // beside it): -2 not measured yet, -1 HIP's copies, else the engine's index; *_rate: GB/s measured
  int d2h_engine = -2, h2d_engine = -2;
  float d2h_rate[8] = {}, h2d_rate[8] = {};
  hsa_agent_t gpu_agent{}, cpu_agent{};
  hsa_signal_t eng_sig[8] = {};

  uint8_t* xbuf(uint64_t bytes);
  uint8_t* sbuf(uint64_t bytes);
  uint8_t* hrows(uint64_t bytes);
  uint8_t* cslow(uint64_t bytes);
};

struct rsk_hll {
  rsk_ctx* ctx = nullptr;
  uint64_t n = 0;
  uint8_t* d_regs = nullptr;   // [n][16384] raw registers (one byte each)
  uint64_t* d_card = nullptr;  // [n] Redis card[8] as LE u64 (bit 63 = cache invalid)
  std::vector<uint8_t> exists; // host: key present
  // host: the key's Redis encoding is dense (HLL_DENSE).  Keys start sparse
  // (createHLLObject); PFMERGE destinations, merged / fetched / all-reduced
  // rows and SET of a dense string are dense; a sparse key is promoted for
  // good once its registers no longer fit the sparse limits (value > 32 or
  // more than hll-sparse-max-bytes = 3000 bytes), checked when it is read out.
  std::vector<uint8_t> dense;
  // Every register is known to be 0 (set by create/clear, dropped by every
  // entry point that may write registers): the grouped add then skips
  // reading the pool.
  mutable bool zero = false;
  // rsk_hll_clear is lazy: the registers are zeroed by the next grouped add
  // that rewrites every row anyway (hll_gapply with write_all), or by
  // hll_materialize before any other access.
  mutable bool pending_clear = false;
  // Part of a lazy clear still pending, per row: after a clear, the routed
  // grouped add (rsk_comm.hip) writes only the rank's owned rows, so every
  // other row keeps its old registers until it is zeroed here (pend[g] = 1:
  // row g reads as cleared; zeroed by hll_materialize, or by
  // hll_materialize_ids / _range for the rows a call touches, or dropped when
  // a row is overwritten whole, as rsk_hll_fetch_rows does).  pending_clear
  // (the whole pool) and pend_n > 0 are never both set.
  mutable std::vector<uint8_t> pend;
  mutable uint64_t pend_n = 0;
  // PFCOUNT precomputed by the partitioned grouped add (hll_gapply estimates
  // every row it writes, from LDS): d_pcount[g] is valid while d_pepoch[g] ==
  // pc_epoch.  Every entry point that may write registers bumps pc_epoch
  // (hll_touch), so a stale estimate is never used; rsk_hll_count takes a
  // valid one instead of re-reading the 16 KiB row, and refreshes the Redis
  // card cache with it exactly as PFCOUNT would.
  uint64_t* d_pcount = nullptr;
  uint32_t* d_pepoch = nullptr;
  mutable uint32_t pc_epoch = 1;
  // rsk_hll_merge_batch leveling state per sketch id (valid while stamp ==
  // lv_epoch): one 12-byte record per sketch, so a pair's lookups touch one
  // cache line per sketch instead of three
  struct Level {
    uint32_t stamp, w, r;
  };
  std::vector<Level> lv;
  uint32_t lv_epoch = 0;
  // SET of a Redis string (rsk_hll_import_redis) keeps the string itself: GET
  // returns those bytes (card bytes as PFCOUNT last left them) until the key is
  // next written, as Redis does -- a canonical re-encoding could chunk the
  // runs of a non-canonical sparse string differently.
  mutable std::unordered_map<uint64_t, std::vector<uint8_t>> imported;
};

struct rsk_bloom {
  rsk_ctx* ctx = nullptr;
  int64_t size = 0;            // bits
  int32_t k = 0;               // hashIterations
  uint64_t nbytes = 0;         // ceil(size/8): the Redis string length
  uint64_t nwords = 0;         // u32 words allocated (>= nbytes/4)
  uint32_t* d_bits = nullptr;  // MSB-first bytes, addressed as LE u32 words
  rsk::FastMod63 fm{};
  // for the RBitSet views of the filter (rsk_bloom_bitset): wgen counts the
  // calls that may have set bits (a view rescans its STRLEN only when it
  // changed), rgen the calls that replaced the whole string (SET: STRLEN =
  // set_len from then on, whatever a view had fixed before)
  uint64_t wgen = 1, rgen = 1, set_len = 0;
};

namespace rsk {

// ---- profiling helpers (rsk_api.hip)
void prof_begin(rsk_ctx* c, const char* name, hipEvent_t* a, hipEvent_t* b);
void prof_end(rsk_ctx* c, const char* name, hipEvent_t a, hipEvent_t b);

struct ProfScope {
  rsk_ctx* c;
  const char* name;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(rsk_ctx* c_, const char* n) : c(c_), name(n) { prof_begin(c, name, &a, &b); }
  ~ProfScope() { prof_end(c, name, a, b); }
};

// Resolved key batch on the device.
struct DevKeys {
  const uint8_t* data;
  const uint64_t* offsets;  // nullptr for fixed stride
  uint64_t n;
  uint32_t fixed_len;
};

// ---- HLL launchers (rsk_hll.hip)
// Adds keys into slabs and max-merges them into sketch `id`; sets *d_flag
// (device u32) to 1 if any register grew.
void hll_add_launch(rsk_ctx* c, const DevKeys& k, uint8_t* d_regs_sketch, uint64_t* d_card, uint32_t* d_flag,
                    uint32_t epoch, bool created);
// Registers of h may change: drop "known zero" and every precomputed PFCOUNT.
void hll_touch(const rsk_hll* h);
// Key id (all keys) written: an imported Redis string is no longer its GET.
inline void hll_forget_import(const rsk_hll* h, uint64_t id) {
  if (!h->imported.empty()) h->imported.erase(id);
}
inline void hll_forget_imports(const rsk_hll* h) { h->imported.clear(); }
struct PCount {  // where hll_gapply leaves its estimates (none: pcount == nullptr)
  uint64_t* pcount;
  uint32_t* pepoch;
  uint32_t epoch;
};
void hll_add_grouped_launch(rsk_ctx* c, const DevKeys& k, const uint32_t* d_groups, uint8_t* d_regs, uint64_t G,
                            bool pool_zero = false, bool write_all = false, PCount pc = PCount{nullptr, nullptr, 0});
// Up to 8 sketch ids passed by value (saves a host->device copy per PFCOUNT).
struct SmallIds {
  uint64_t v[8];
  uint32_t n;
};
void hll_count_launch(rsk_ctx* c, const uint8_t* d_regs, uint64_t* d_card, const uint64_t* d_ids,
                      const SmallIds& small, uint64_t n, uint64_t* d_out, PCount pc = PCount{nullptr, nullptr, 0});
void hll_union_count_launch(rsk_ctx* c, const uint8_t* const* d_member_ptrs, uint32_t arity, uint64_t n,
                            uint64_t* d_out);
void hll_merge_launch(rsk_ctx* c, uint8_t* const* d_dst_ptrs, const uint8_t* const* d_src_ptrs, uint32_t srcs_per_dst,
                      uint64_t n);
void hll_add_each_launch(rsk_ctx* c, const DevKeys& k, const uint8_t* d_regs_sketch, uint8_t* d_out);
void hll_max_into_launch(rsk_ctx* c, uint8_t* d_dst, const uint8_t* d_src, uint32_t* d_flag);

// ---- Redis strings of many keys (rsk_hll_io.hip)
// Export: key d_ids[i]'s string encoded into d_slots + i * 12304 and its
// length in d_len[i] (bit 31: sparse; d_want_sparse[i]: the key is still in
// the sparse encoding); pack: string i from its slot to d_out + d_pos[i].
void hll_export_launch(rsk_ctx* c, const uint8_t* d_regs, const uint64_t* d_card, const uint64_t* d_ids,
                       const uint8_t* d_want_sparse, uint32_t n, uint32_t* d_len, uint8_t* d_slots);
void hll_export_pack_launch(rsk_ctx* c, const uint8_t* d_slots, const uint32_t* d_len, const uint64_t* d_pos,
                            uint32_t n, uint8_t* d_out);
// Import: d_apply null -> check the sparse strings (atomicMin(d_err, i0 + i)
// on a corrupt one; d_canon[i] = 0 where the payload is not the canonical
// encoding); d_apply given -> decode strings with d_apply[i] set into rows
// d_ids[i] (and their card bytes), unless *d_err was set.  A call may check
// its strings in chunks (pointers advanced by the chunk's first string i0).
void hll_import_launch(rsk_ctx* c, const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_ids,
                       const uint8_t* d_apply, uint32_t n, uint8_t* d_regs, uint64_t* d_card, uint8_t* d_canon,
                       unsigned long long* d_err, uint32_t i0 = 0);
// The rows (and card words) strings i with d_apply[i] will replace, copied to
// d_bak row i (restore = false), or copied back if *d_err is set (restore).
void hll_rows_bak_launch(rsk_ctx* c, bool restore, uint8_t* d_regs, uint64_t* d_card, const uint64_t* d_ids,
                         const uint8_t* d_apply, uint32_t n, uint8_t* d_bak, uint64_t* d_bak_card,
                         const unsigned long long* d_err);

// ---- Bloom launchers (rsk_bloom.hip)
void bloom_add_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k);
// Slice-partitioned add (rsk_bloom_part.hip); false when the direct kernel is used
// (small batch, k > 4096, filter > 2^34 bits, or RSK_BLOOM_PARTITION=0).
bool bloom_add_partitioned(rsk_ctx* c, rsk_bloom* b, const DevKeys& k);
// Super-tile partition (rsk_bloom_st.hip); false when not applicable (small
// batch, k > 16, filter > 2^34 bits, or RSK_BLOOM_ST=0).
bool bloom_add_supertile(rsk_ctx* c, rsk_bloom* b, const DevKeys& k);
void bloom_add_direct_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k);
// Grouped PFADD partitioned by sketch (rsk_bloom_part.hip); false when the
// batch is not worth it (or not 16-byte keys): use the direct kernel.
bool hll_grouped_partition_applies(const rsk_ctx* c, const DevKeys& k, uint64_t G, bool recs = false);
// d_recs: the input is already hashed (8-byte records {group, index << 6 | rank}, k.n of them)
bool hll_add_grouped_partitioned(rsk_ctx* c, const DevKeys& k, const uint32_t* d_groups, uint8_t* d_regs, uint64_t G,
                                 bool pool_zero, bool write_all, PCount pc, const uint2* d_recs = nullptr);
// Owner-routed grouped add (rsk_hll_group.hip; the exchange in rsk_comm.hip):
// per-block owner counts cnt[o * B + b] (B = route_blocks), then the pairs
// hashed into 8-byte records appended to owner o's run at off[o * B + b].
uint32_t route_blocks(const rsk_ctx* c);
void hll_route_count_launch(rsk_ctx* c, const uint32_t* d_groups, uint64_t n, uint64_t G, uint32_t N,
                            const uint32_t* d_slot_of, const uint32_t* d_hbits, uint32_t* d_cnt);
void hll_route_scatter_launch(rsk_ctx* c, const uint8_t* d_keys16, const uint32_t* d_groups, uint64_t n, uint64_t G,
                              uint32_t N, const uint32_t* d_slot_of, const uint32_t* d_hbits, const uint64_t* d_off,
                              uint2* d_out);
// Heavy groups of a routed add (skew): sampled counts (every stride-th pair), a
// group is heavy when its sample count reaches thr and it lies outside
// [skip_lo, skip_hi); at most cap, by group id.
// scratch: hll_heavy_scratch_bytes(G, cap) of device memory; *d_slot_of points
// into it (a group's slot, ~0 if light), *d_hbits to the bitmap of the heavy
// groups, heavy_ids gets the heavy groups ascending (slot order).  Returns
// their number; synchronises the stream.
uint64_t hll_heavy_scratch_bytes(uint64_t G, uint32_t cap);
uint64_t hll_heavy_select(rsk_ctx* c, const uint32_t* d_groups, uint64_t n, uint64_t G, uint32_t stride, uint32_t thr,
                          uint64_t skip_lo, uint64_t skip_hi, uint32_t cap, uint8_t* scratch, uint32_t** d_slot_of,
                          uint32_t** d_hbits, std::vector<uint32_t>* heavy_ids);
// Records into a pool of G rows (partitioned for large batches, else a CAS each);
// write_all: every row written (zero rows for sketches without records).
void hll_add_grouped_recs_launch(rsk_ctx* c, const uint2* d_recs, uint64_t n, uint8_t* d_regs, uint64_t G,
                                 bool pool_zero, bool write_all, PCount pc);
// Performs a pending lazy clear (rsk_api.hip).
void hll_materialize(const rsk_hll* h);
// The rows among ids[0..n) / [first, first + count) that a partial lazy clear
// left pending are zeroed (and the stream synchronised); a whole-pool pending
// clear is completed as by hll_materialize.
void hll_materialize_ids(const rsk_hll* h, const uint64_t* ids, uint64_t n);
void hll_materialize_range(const rsk_hll* h, uint64_t first, uint64_t count);
// Rows [first, first + count) hold data, every other row is pending clear.
void hll_pend_outside(const rsk_hll* h, uint64_t first, uint64_t count);
// Rows overwritten whole (no longer pending).
void hll_unpend(const rsk_hll* h, const uint64_t* ids, uint64_t n);
void bloom_add_each_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
// add() replies (RedissonBloomFilter.java:100-107) + the insert, any batch size:
// the partitioned first-probe pipeline (rsk_bloom_reply.hip) when it applies,
// else the sort path in sub-batches of 2^28 probes.
void bloom_add_replies_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
void bloom_add_replies_sorted(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
bool bloom_add_replies_append(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
void bloom_contains_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
void bloom_bitcount_launch(rsk_ctx* c, const uint32_t* d_bits, uint64_t nwords, uint64_t* d_out);
// misc/Hash.hashToBase64 of every key: 22 chars per key into d_out.
void hash_b64_launch(rsk_ctx* c, const DevKeys& k, char* d_out);
void bloom_or_launch(rsk_ctx* c, uint32_t* d_bits, const uint8_t* d_src, uint64_t nbytes);
// dst[0..words) |= OR over rows of src (row r at src + r*stride words; stride
// and dst 16-byte aligned, words any count).
void or_rows_into_launch(rsk_ctx* c, uint32_t* d_dst, const uint32_t* d_src, uint32_t rows, uint64_t words,
                         uint64_t stride);

// ---- exchange plans (rsk_plan.hip, host only)
void plan_owned_range(uint64_t n, uint64_t N, uint64_t r, uint64_t* first, uint64_t* count);
uint64_t plan_owner(uint64_t n, uint64_t N, uint64_t id);
uint64_t plan_bloom_slice_words(uint64_t nwords, uint64_t N);
bool plan_fetch(uint64_t n, uint64_t N, uint64_t r, const uint64_t* ids, uint64_t n_ids, uint32_t flags,
                std::vector<uint64_t>* want, std::vector<uint64_t>* counts);
void plan_heavy_rows(uint64_t G, uint64_t N, const uint32_t* heavy_ids, uint64_t H, std::vector<uint64_t>* rows);

}  // namespace rsk
