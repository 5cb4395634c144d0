/*
 * rsk_oracle.h -- CPU restatement of the sketch arithmetic behind Redisson's
 * RHyperLogLog / RBloomFilter / RBitSet path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path (redisson_amd + librsketch.so) never links or calls it.
 *
 * The arithmetic on this path lives outside /root/reference:
 *   - Redis 3.2.0 src/hyperloglog.c  (pinned by .travis.yml:24 of the reference):
 *       MurmurHash64A, hllPatLen, dense/sparse encodings, hllCount, PFMERGE.
 *   - Redis 3.2.0 src/bitops.c: SETBIT/GETBIT/BITCOUNT MSB-first addressing.
 *   - net.openhft:zero-allocation-hashing 0.5 (reference pom.xml:226-230):
 *       LongHashFunction.xx_r39() = XXH64 seed 0, farmUo() = farmhash 1.1
 *       farmhashuo::Hash64 (== farmhashna::Hash64 for len <= 64).
 * Each function below names the upstream routine it restates and the
 * reference call site that reaches it.  Pinning: see oracle/README.md.
 */
#ifndef RSK_ORACLE_H
#define RSK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_HLL_P 14
#define ORC_HLL_REGISTERS 16384
#define ORC_HLL_BITS 6
#define ORC_HLL_HDR_SIZE 16
#define ORC_HLL_DENSE_SIZE (ORC_HLL_HDR_SIZE + (ORC_HLL_REGISTERS * ORC_HLL_BITS + 7) / 8)

/* ---- hashes ---------------------------------------------------------- */
uint64_t orc_murmur64a(const void *key, int len, uint32_t seed);
uint64_t orc_xxh64(const void *key, size_t len, uint64_t seed);
uint64_t orc_farmhash_na64(const void *key, size_t len);
uint64_t orc_farmhash_uo64(const void *key, size_t len);
uint64_t orc_splitmix64(uint64_t x);

/* ---- HyperLogLog (Redis 3.2.0) -------------------------------------- */
int orc_hll_patlen(const uint8_t *ele, size_t len, long *regp);
/* PFADD arithmetic on raw (one byte per register) registers; returns the
 * number of registers that grew. */
void orc_hll_records(const uint8_t *data, uint32_t fixed_len, uint64_t n, uint32_t *out);
uint64_t orc_hll_add_raw(uint8_t *regs, const uint8_t *data, const uint64_t *offsets,
                         uint32_t fixed_len, uint64_t n);
/* Fixed-length keys on nthreads cores (OpenMP, private registers, max-merge). */
void orc_hll_add_fixed_mt(uint8_t *regs, const uint8_t *data, uint32_t fixed_len, uint64_t n, int nthreads);
/* Same, but the keys are the synthetic 16-byte stream of SURVEY 8d (C2),
 * generated on the fly; nthreads > 1 uses OpenMP with private registers. */
void orc_hll_add_gen16(uint8_t *regs, uint64_t seed, uint64_t start, uint64_t n, int nthreads);
/* The C4 variable-length stream (8-64 B keys), generated on the fly. */
void orc_hll_add_gen_varlen(uint8_t *regs, uint64_t seed, uint64_t start, uint64_t n, int nthreads);
/* Grouped variant (C5 stream): regs is [G][16384]. */
void orc_hll_add_gen_grouped(uint8_t *regs, uint64_t G, uint64_t seed, uint64_t start, uint64_t n);
/* Groups [0, gsub) only (regs is [gsub][16384]), on nthreads cores. */
void orc_hll_add_gen_grouped_subset(uint8_t *regs, uint64_t G, uint64_t gsub, uint64_t seed, uint64_t start,
                                    uint64_t n, int nthreads);
/* Groups ids[0..nids) (distinct), regs [nids][16384], on nthreads cores. */
void orc_hll_add_gen_grouped_ids(uint8_t *regs, uint64_t G, const uint64_t *ids, uint64_t nids, uint64_t seed,
                                 uint64_t start, uint64_t n, int nthreads);

int orc_hll_dense_get(const uint8_t *dense_regs, int j);
void orc_hll_dense_set(uint8_t *dense_regs, int j, int v);
double orc_hll_dense_sum(const uint8_t *dense_regs, int *ezp);
double orc_hll_raw_sum(const uint8_t *raw_regs, int *ezp);
double orc_hll_sparse_sum(const uint8_t *sparse, int sparselen, int *ezp, int *invalid);
uint64_t orc_hll_estimate(double E, int ez);
uint64_t orc_hll_count_raw(const uint8_t *raw_regs);
uint64_t orc_hll_count_dense_regs(const uint8_t *raw_regs);
/* Redis string encodings. */
int orc_hll_encode_dense(const uint8_t *raw_regs, const uint8_t card[8], uint8_t *out, size_t cap);
int orc_hll_encode_sparse(const uint8_t *raw_regs, const uint8_t card[8], uint8_t *out, size_t cap);
int orc_hll_decode(const uint8_t *buf, size_t len, uint8_t *raw_regs, int *encoding);
/* PFCOUNT on a stored Redis string (honours the cached cardinality). */
int orc_hll_count_string(const uint8_t *buf, size_t len, uint64_t *out);

/* ---- Bloom filter (RedissonBloomFilter.java) ------------------------- */
int64_t orc_bloom_optimal_bits(int64_t n, double p);
int32_t orc_bloom_optimal_k(int64_t n, int64_t m);
void orc_bloom_indexes(const uint8_t *key, size_t len, int k, int64_t size, int64_t *out);
int32_t orc_bloom_count(int64_t size, int k, int64_t bitcount);
/* Sequential (input-order) add/contains over an MSB-first bitset of
 * ceil(size/8) bytes; added_out/out may be NULL. */
void orc_bloom_add_batch(uint8_t *bits, int64_t size, int k, const uint8_t *data,
                         const uint64_t *offsets, uint32_t fixed_len, uint64_t n, uint8_t *added_out);
void orc_bloom_contains_batch(const uint8_t *bits, int64_t size, int k, const uint8_t *data,
                              const uint64_t *offsets, uint32_t fixed_len, uint64_t n, uint8_t *out);

/* The C3 streams on nthreads cores (full-size parity checks). */
void orc_bloom_add_gen16_mt(uint8_t *bits, int64_t size, int k, uint64_t seed, uint64_t start, uint64_t n,
                            int nthreads);
uint64_t orc_bloom_contains_gen_queries_mt(const uint8_t *bits, int64_t size, int k, uint64_t qseed, uint64_t iseed,
                                           uint64_t n_ins, uint64_t start, uint64_t n, uint8_t *out, int nthreads);
/* add() replies of the sampled keys sample[0..ns) when keys 0..n-1 of the C3
 * stream are added in one batch to an empty filter. */
void orc_bloom_add_replies_sample_gen16_mt(int64_t size, int k, uint64_t seed, uint64_t n, const uint64_t *sample,
                                           uint64_t ns, uint8_t *out, int nthreads);

/* ---- Redis bitops (MSB-first string) -------------------------------- */
int orc_setbit(uint8_t *bits, uint64_t off, int v);
int orc_getbit(const uint8_t *bits, uint64_t off);
uint64_t orc_bitcount(const uint8_t *bits, uint64_t nbytes);

/* ---- synthetic inputs ------------------------------------ */
void orc_gen_keys16(uint64_t seed, uint64_t start, uint64_t n, uint8_t *out);
uint32_t orc_gen_varlen_len(uint64_t seed, uint64_t i);
void orc_gen_varlen_key(uint64_t seed, uint64_t i, uint8_t *out);
void orc_gen_grouped(uint64_t seed, uint64_t G, uint64_t start, uint64_t n, uint32_t *groups, uint8_t *keys);
void orc_zipf_cdf(uint64_t G, double s, uint64_t *cdf);
void orc_gen_grouped_zipf(uint64_t seed, uint64_t G, double s, uint64_t start, uint64_t n, uint32_t *groups,
                          uint8_t *keys);
void orc_hll_add_gen_grouped_zipf_subset(uint8_t *regs, uint64_t G, uint64_t gsub, double s, uint64_t seed,
                                         uint64_t start, uint64_t n, int nthreads);
void orc_gen_queries16(uint64_t qseed, uint64_t iseed, uint64_t n_ins, uint64_t start, uint64_t n, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
