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

// Heavy rows of a routed add per owner: heavy_ids ascending (the slot order),
// so owner o's rows are the slots [sum of rows[< o], + rows[o]).
void plan_heavy_rows(uint64_t G, uint64_t N, const uint32_t* heavy_ids, uint64_t H, std::vector<uint64_t>* rows) {
  rows->assign(N, 0);
  for (uint64_t i = 0; i < H; ++i) ++(*rows)[plan_owner(G, N, heavy_ids[i])];
}

// The routed grouped add's traffic per owner (rsk_hll_add_grouped_routed): from
// counts[s * G + g] = pairs of group g on source rank s, with the groups of at
// least heavy_min pairs owned by another rank (0: none; at most heavy_cap per
// source, lowest ids first) pre-combined at the source into one 16 KiB row each.  Per rank o:
// bytes received from the other ranks (8 B per light record, 16384 + 4 B per
// heavy row and its id), heavy rows received, and light records its apply
// folds (its own included).  The device takes the heavy set from a sampled
// count (every stride-th pair) instead of the exact one.
void plan_route_recv(const uint64_t* counts, uint64_t G, uint64_t N, uint64_t heavy_min, uint64_t heavy_cap,
                     uint64_t* recv_bytes, uint64_t* recv_rows, uint64_t* apply_records) {
  for (uint64_t o = 0; o < N; ++o) recv_bytes[o] = recv_rows[o] = apply_records[o] = 0;
  for (uint64_t s = 0; s < N; ++s) {
    const uint64_t* cs = counts + s * G;
    uint64_t heavy = 0;
    for (uint64_t g = 0; g < G; ++g) {
      const uint64_t k = cs[g];
      if (!k) continue;
      const uint64_t o = plan_owner(G, N, g);
      if (heavy_min && k >= heavy_min && o != s && heavy < heavy_cap) {
        ++heavy;
        if (o != s) {
          recv_bytes[o] += 16384 + 4;
          ++recv_rows[o];
        }
      } else {
        apply_records[o] += k;
        if (o != s) recv_bytes[o] += 8 * k;
      }
    }
  }
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

int rsk_plan_route_recv(const uint64_t* counts, uint64_t G, int nranks, uint64_t heavy_min, uint64_t heavy_cap,
                        uint64_t* recv_bytes, uint64_t* recv_rows, uint64_t* apply_records) {
  if (nranks < 1 || (!counts && G) || !recv_bytes || !recv_rows || !apply_records) return RSK_ERR_INVALID_ARG;
  rsk::plan_route_recv(counts, G, (uint64_t)nranks, heavy_min, heavy_cap, recv_bytes, recv_rows, apply_records);
  return RSK_OK;
}

}  // extern "C"
