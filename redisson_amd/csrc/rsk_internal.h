// rsk_internal.h -- host-side internals shared by the librsketch translation
// units (context, handles, error plumbing, kernel launchers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsketch.h"
#include "../../include/rsketch_diag.h"
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
  // double-buffered pinned host stages (filled by host threads while the
  // previous chunk's DMA runs), their device twins and "DMA done" events;
  // pin_off: pinned allocation failed, copy from the pageable source
  uint8_t* h_pin[2] = {nullptr, nullptr};
  uint8_t* d_pin[2] = {nullptr, nullptr};
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
  bool pin_off = false;
  // per-workgroup partial register files [slabs][16384] u8
  uint8_t* d_slab = nullptr;
  uint32_t slab_count = 0;
  // small scratch: flags / counters / ids (device) and pinned host mirror
  uint8_t* d_small = nullptr;
  uint8_t* h_small = nullptr;
  uint64_t small_bytes = 0;
  // grow-on-demand device scratch for batched calls
  uint8_t* d_work = nullptr;
  uint64_t work_bytes = 0;
  // grow-on-demand pinned host scratch: per-op arrays of batched calls
  // (countWith / mergeWith sketch pointers) built in place and copied with
  // one asynchronous DMA; a call that returns before its DMA has run (the
  // reply-less rsk_hll_merge_batch) records batch_ev, and pinned() waits for
  // it before the buffer is written again
  uint8_t* h_batch = nullptr;
  uint64_t h_batch_bytes = 0;
  hipEvent_t batch_ev = nullptr;
  bool batch_pending = false;
  // m*log(m/ez) for ez = 0..16384, computed with the host libm (Redis's log)
  double* d_lc = nullptr;
  rsk::Profiler prof;
  // RCCL communicator (multi-GPU merge layer), null when single-GPU
  void* comm = nullptr;
  int nranks = 1;
  int rank = 0;
  // call number written by kernels that report "something changed" (no reset)
  uint32_t epoch = 0;

  uint8_t* work(uint64_t bytes);
  uint8_t* pinned(uint64_t bytes);
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
};

struct rsk_bloom {
  rsk_ctx* ctx = nullptr;
  int64_t size = 0;            // bits
  int32_t k = 0;               // hashIterations
  uint64_t nbytes = 0;         // ceil(size/8): the Redis string length
  uint64_t nwords = 0;         // u32 words allocated (>= nbytes/4)
  uint32_t* d_bits = nullptr;  // MSB-first bytes, addressed as LE u32 words
  rsk::FastMod63 fm{};
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
void hll_variant_launch(rsk_ctx* c, int variant, const uint4* keys, uint64_t n);
// Blob+offsets PFADD variants (rsk_diag_hll_var_variant), slabs only.
void hll_var_variant_launch(rsk_ctx* c, int variant, const uint8_t* data, const uint64_t* offsets, uint64_t n);

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
bool hll_grouped_partition_applies(const DevKeys& k, uint64_t G);
bool hll_add_grouped_partitioned(rsk_ctx* c, const DevKeys& k, const uint32_t* d_groups, uint8_t* d_regs, uint64_t G,
                                 bool pool_zero, bool write_all, PCount pc);
// Performs a pending lazy clear (rsk_api.hip).
void hll_materialize(const rsk_hll* h);
void bloom_add_each_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
// add() replies (RedissonBloomFilter.java:100-107) + the insert, any batch size:
// the partitioned first-probe pipeline (rsk_bloom_reply.hip) when it applies,
// else the sort path in sub-batches of 2^28 probes.
void bloom_add_replies_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
void bloom_add_replies_sorted(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
bool bloom_add_replies_append(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
void bloom_contains_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out);
void bloom_contains_variant_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out, int variant);
void bloom_contains_probe_count_launch(rsk_ctx* c, rsk_bloom* b, const DevKeys& k, uint8_t* d_out,
                                       unsigned long long* d_probes);
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

// ---- generators (rsk_gen.hip)
void gen_keys16_launch(rsk_ctx* c, uint64_t seed, uint64_t start, uint64_t n, void* out);
void gen_grouped_launch(rsk_ctx* c, uint64_t seed, uint64_t G, uint64_t start, uint64_t n, uint32_t* g, void* keys);
std::vector<uint64_t> zipf_cdf(uint32_t G, double s);
void gen_grouped_zipf_launch(rsk_ctx* c, uint64_t seed, const uint64_t* d_cdf, uint32_t G, uint64_t start, uint64_t n,
                             uint32_t* g, void* keys);
void gen_queries16_launch(rsk_ctx* c, uint64_t qseed, uint64_t iseed, uint64_t n_ins, uint64_t start, uint64_t n,
                          void* out);
void gen_varlen_lengths_launch(rsk_ctx* c, uint64_t seed, uint64_t start, uint64_t n, uint64_t* offsets);
void gen_varlen_bytes_launch(rsk_ctx* c, uint64_t seed, uint64_t start, uint64_t n, const uint64_t* offsets,
                             uint8_t* blob);

}  // namespace rsk
