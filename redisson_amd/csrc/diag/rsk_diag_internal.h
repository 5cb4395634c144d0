// rsk_diag_internal.h -- the test and bench support library
// (librsketch_diag.so, include/rsketch_diag.h).  It is built from the same
// internal headers as librsketch.so, so it sees a context's layout (stream,
// scratch, route overrides) without the product library exporting anything
// beyond its C ABI; it never calls into the product library's internals.
#pragma once
#include <string>

#include "../../../include/rsketch_diag.h"
#include "../rsk_internal.h"

namespace rsk {
namespace diag {
void set_error(const std::string& msg);

template <class F>
int guarded(F&& fn) {
  try {
    fn();
    set_error("");
    return RSK_OK;
  } catch (const RskError& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_error(e.what());
    return RSK_ERR_DEVICE;
  }
}

inline void need(bool cond, const char* msg) {
  if (!cond) throw RskError{RSK_ERR_INVALID_ARG, msg};
}

struct Lock {
  std::lock_guard<std::recursive_mutex> g;
  explicit Lock(rsk_ctx* c) : g(c->mu) { RSK_HIP(hipSetDevice(c->device)); }
};
}  // namespace diag

// tuning variants and tallies (rsk_diag_kernels.hip)
void hll_variant_launch(rsk_ctx* c, int variant, const uint4* keys, uint64_t n);
void hll_var_variant_launch(rsk_ctx* c, int variant, const uint8_t* data, const uint64_t* offsets, uint64_t n);
void bloom_contains_variant_launch(rsk_ctx* c, rsk_bloom* b, const uint4* keys, uint64_t n, uint8_t* d_out,
                                   int variant);
void bloom_contains_probe_count_launch(rsk_ctx* c, rsk_bloom* b, const uint4* keys, uint64_t n, uint8_t* d_out,
                                       unsigned long long* d_probes);

// generators (rsk_gen.hip)
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
