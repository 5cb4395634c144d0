// rsk_plan.hip -- host-only arithmetic of the multi-GPU exchange plans.
//
// rsk_comm.hip runs these plans over RCCL; they are exported on their own
// (include/rsketch.h, "exchange plans") so the N > 1 arithmetic is testable
// without GPUs: tests/test_plan.py checks them against redisson_amd/shard.py,
// whose restatement the gloo tests run at world sizes 2 and 3, and the
// sanitizer build (oracle/Makefile `asan`) runs them under ASan/UBSan.
//
// No HIP API is used here (compiles as plain C++: g++ -x c++).
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../../include/rsketch.h"

namespace rsk {

// Key-stream sharding (ShardPlan.range): the first n mod world ranks get one
// key more, ranges are contiguous and ascending by rank.
void plan_shard_range(uint64_t n, uint64_t world, uint64_t rank, uint64_t* begin, uint64_t* end) {
  const uint64_t base = n / world, extra = n % world;
  *begin = rank * base + std::min(rank, extra);
  *end = *begin + base + (rank < extra ? 1 : 0);
}

// Owned sketches after the MAX reduce-scatter of a pool of n sketches:
// rank r owns [r*q, (r+1)*q), q = n / N; the last rank also owns the n mod N tail.
void plan_owned_range(uint64_t n, uint64_t N, uint64_t r, uint64_t* first, uint64_t* count) {
  const uint64_t q = n / N;
  *first = r * q;
  *count = q + (r == N - 1 ? n - q * N : 0);
}

uint64_t plan_owner(uint64_t n, uint64_t N, uint64_t id) {
  const uint64_t q = n / N;
  return q ? std::min<uint64_t>(id / q, N - 1) : N - 1;
}

// Bloom slice-OR: S words per rank, a multiple of 4 (16-byte vector OR), N*S >= nwords.
uint64_t plan_bloom_slice_words(uint64_t nwords, uint64_t N) {
  uint64_t S = (nwords + N - 1) / N;
  return (S + 3) & ~uint64_t(3);
}

// rsk_hll_fetch_rows request plan: the distinct ids this rank needs from
// others, ascending (hence grouped by owner), and how many go to each owner.
// With RSK_FETCH_SELF the ids this rank owns are requested too (from itself).
// Returns false if an id is outside the pool (want/counts are then empty).
bool plan_fetch(uint64_t n, uint64_t N, uint64_t r, const uint64_t* ids, uint64_t n_ids, uint32_t flags,
                std::vector<uint64_t>* want, std::vector<uint64_t>* counts) {
  want->assign(ids, ids + n_ids);
  counts->assign(N, 0);
  for (uint64_t id : *want)
    if (id >= n) {
      want->clear();
      return false;
    }
  std::sort(want->begin(), want->end());
  want->erase(std::unique(want->begin(), want->end()), want->end());
  if (!(flags & RSK_FETCH_SELF))
    want->erase(std::remove_if(want->begin(), want->end(), [&](uint64_t id) { return plan_owner(n, N, id) == r; }),
                want->end());
  for (uint64_t id : *want) ++(*counts)[plan_owner(n, N, id)];
  return true;
}

}  // namespace rsk

extern "C" {

int rsk_plan_shard_range(uint64_t n, int world, int rank, uint64_t* begin, uint64_t* end) {
  if (world < 1 || rank < 0 || rank >= world || !begin || !end) return RSK_ERR_INVALID_ARG;
  rsk::plan_shard_range(n, (uint64_t)world, (uint64_t)rank, begin, end);
  return RSK_OK;
}

int rsk_plan_owned_range(uint64_t n, int nranks, int rank, uint64_t* first, uint64_t* count) {
  if (nranks < 1 || rank < 0 || rank >= nranks || !first || !count) return RSK_ERR_INVALID_ARG;
  rsk::plan_owned_range(n, (uint64_t)nranks, (uint64_t)rank, first, count);
  return RSK_OK;
}

int rsk_plan_owner(uint64_t n, int nranks, uint64_t id, int* owner) {
  if (nranks < 1 || !owner || id >= n) return RSK_ERR_INVALID_ARG;
  *owner = (int)rsk::plan_owner(n, (uint64_t)nranks, id);
  return RSK_OK;
}

int rsk_plan_bloom_slice_words(uint64_t nwords, int nranks, uint64_t* words) {
  if (nranks < 1 || !words) return RSK_ERR_INVALID_ARG;
  *words = rsk::plan_bloom_slice_words(nwords, (uint64_t)nranks);
  return RSK_OK;
}

int rsk_plan_fetch(uint64_t n, int nranks, int rank, const uint64_t* ids, uint64_t n_ids, uint32_t flags,
                   uint64_t* want_out, uint64_t* n_want, uint64_t* counts_out) {
  if (nranks < 1 || rank < 0 || rank >= nranks || (!ids && n_ids) || !n_want || !counts_out ||
      (!want_out && n_ids))
    return RSK_ERR_INVALID_ARG;
  std::vector<uint64_t> want, counts;
  if (!rsk::plan_fetch(n, (uint64_t)nranks, (uint64_t)rank, ids, n_ids, flags, &want, &counts))
    return RSK_ERR_INVALID_ARG;
  std::copy(want.begin(), want.end(), want_out);
  std::copy(counts.begin(), counts.end(), counts_out);
  *n_want = want.size();
  return RSK_OK;
}

}  // extern "C"
