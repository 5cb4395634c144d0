/*
 * rsk_oracle.c -- CPU restatement (checker) of the sketch arithmetic on the
 * Redisson HLL / Bloom / BitSet path.  TEST INFRASTRUCTURE ONLY: see the
 * header comment in rsk_oracle.h.  Compiled with -ffp-contract=off so the
 * FP64 estimator matches Redis built by gcc -O2 on x86-64 (no FMA).
 *
 * Upstream routines restated here (not present in /root/reference):
 *   Redis 3.2.0 src/hyperloglog.c, src/bitops.c;
 *   xxHash XXH64 (OpenHFT xx_r39), farmhash 1.1 farmhashna / farmhashuo.
 * Reference call sites: RedissonHyperLogLog.java:65-97 (PFADD/PFCOUNT/PFMERGE),
 * RedissonBloomFilter.java:69-78,116-131,188-199, RedissonBitSet.java:152-173.
 */
#include "rsk_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline uint64_t ld64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v; /* x86-64 host: little-endian, as Redis and OpenHFT read */
}
static inline uint32_t ld32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint64_t rotr64(uint64_t v, int s) { return s == 0 ? v : (v >> s) | (v << (64 - s)); }
static inline uint64_t rotl64(uint64_t v, int s) { return s == 0 ? v : (v << s) | (v >> (64 - s)); }

/* ===================================================================== */
/* Redis 3.2.0 hyperloglog.c: MurmurHash64A (used by hllPatLen).          */
/* ===================================================================== */
uint64_t orc_murmur64a(const void *key, int len, uint32_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ULL;
    const int r = 47;
    uint64_t h = (uint64_t)seed ^ ((uint64_t)(int64_t)len * m);
    const uint8_t *data = (const uint8_t *)key;
    const uint8_t *end = data + (len - (len & 7));
    while (data != end) {
        uint64_t k = ld64(data);
        k *= m;
        k ^= k >> r;
        k *= m;
        h ^= k;
        h *= m;
        data += 8;
    }
    switch (len & 7) {
    case 7: h ^= (uint64_t)data[6] << 48; /* fall through */
    case 6: h ^= (uint64_t)data[5] << 40; /* fall through */
    case 5: h ^= (uint64_t)data[4] << 32; /* fall through */
    case 4: h ^= (uint64_t)data[3] << 24; /* fall through */
    case 3: h ^= (uint64_t)data[2] << 16; /* fall through */
    case 2: h ^= (uint64_t)data[1] << 8;  /* fall through */
    case 1: h ^= (uint64_t)data[0]; h *= m;
    }
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}

/* Redis 3.2.0 hllPatLen: index = low 14 bits, rank = 1 + run of zeros from
 * bit 14 upward, bit 63 forced so the rank is at most 50. */
int orc_hll_patlen(const uint8_t *ele, size_t len, long *regp) {
    uint64_t hash = orc_murmur64a(ele, (int)len, 0xadc83b19U);
    uint64_t index = hash & (ORC_HLL_REGISTERS - 1);
    uint64_t bit = ORC_HLL_REGISTERS;
    int count = 1;
    hash |= (uint64_t)1 << 63;
    while ((hash & bit) == 0) {
        count++;
        bit <<= 1;
    }
    *regp = (long)index;
    return count;
}

/* The (register index, rank) of each fixed-length key as index << 6 | rank:
 * the record the owner-routed grouped add ships (rsk_hll_add_grouped_routed),
 * from hllPatLen above. */
void orc_hll_records(const uint8_t *data, uint32_t fixed_len, uint64_t n, uint32_t *out) {
    for (uint64_t i = 0; i < n; i++) {
        long idx;
        const int c = orc_hll_patlen(data + i * (uint64_t)fixed_len, fixed_len, &idx);
        out[i] = ((uint32_t)idx << 6) | (uint32_t)c;
    }
}

uint64_t orc_hll_add_raw(uint8_t *regs, const uint8_t *data, const uint64_t *offsets,
                         uint32_t fixed_len, uint64_t n) {
    uint64_t grown = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p;
        size_t len;
        if (offsets) {
            p = data + offsets[i];
            len = (size_t)(offsets[i + 1] - offsets[i]);
        } else {
            p = data + i * (uint64_t)fixed_len;
            len = fixed_len;
        }
        long idx;
        int c = orc_hll_patlen(p, len, &idx);
        if (c > regs[idx]) {
            regs[idx] = (uint8_t)c;
            grown++;
        }
    }
    return grown;
}

/* The same over fixed-length keys on nthreads host cores: OpenMP, private
 * registers per thread, max-merged at the end (SURVEY 8d's "all host cores"
 * CPU figure; registers equal orc_hll_add_raw's because max commutes). */
void orc_hll_add_fixed_mt(uint8_t *regs, const uint8_t *data, uint32_t fixed_len, uint64_t n, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 1) {
        uint8_t *priv = (uint8_t *)calloc((size_t)nthreads, ORC_HLL_REGISTERS);
#pragma omp parallel num_threads(nthreads)
        {
            uint8_t *mine = priv + (size_t)omp_get_thread_num() * ORC_HLL_REGISTERS;
#pragma omp for schedule(static)
            for (uint64_t i = 0; i < n; i++) {
                long idx;
                int c = orc_hll_patlen(data + i * (uint64_t)fixed_len, fixed_len, &idx);
                if (c > mine[idx]) mine[idx] = (uint8_t)c;
            }
        }
        for (int t = 0; t < nthreads; t++)
            for (int j = 0; j < ORC_HLL_REGISTERS; j++)
                if (priv[(size_t)t * ORC_HLL_REGISTERS + j] > regs[j]) regs[j] = priv[(size_t)t * ORC_HLL_REGISTERS + j];
        free(priv);
        return;
    }
#endif
    (void)nthreads;
    orc_hll_add_raw(regs, data, NULL, fixed_len, n);
}

/* ===================================================================== */
/* Synthetic inputs.  splitmix64 output for state x.          */
/* ===================================================================== */
uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_gen_keys16(uint64_t seed, uint64_t start, uint64_t n, uint8_t *out) {
    for (uint64_t j = 0; j < n; j++) {
        uint64_t i = start + j;
        uint64_t lo = orc_splitmix64(seed + 2 * i), hi = orc_splitmix64(seed + 2 * i + 1);
        memcpy(out + 16 * j, &lo, 8);
        memcpy(out + 16 * j + 8, &hi, 8);
    }
}

uint32_t orc_gen_varlen_len(uint64_t seed, uint64_t i) {
    return 8u + (uint32_t)(orc_splitmix64(seed ^ i) % 57u);
}

void orc_gen_varlen_key(uint64_t seed, uint64_t i, uint8_t *out) {
    uint32_t len = orc_gen_varlen_len(seed, i);
    for (uint32_t w = 0; w * 8 < len; w++) {
        uint64_t r = orc_splitmix64(seed + (i << 3) + w);
        for (uint32_t b = 0; b < 8 && w * 8 + b < len; b++)
            out[w * 8 + b] = (uint8_t)(0x21 + ((r >> (8 * b)) & 0xFF) % 94);
    }
}

/* PFADD arithmetic over the C4 stream generated on the fly (keys start ..
 * start+n-1); nthreads > 1 uses OpenMP with private registers + max-merge. */
void orc_hll_add_gen_varlen(uint8_t *regs, uint64_t seed, uint64_t start, uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    uint8_t *priv = (uint8_t *)calloc((size_t)nthreads, ORC_HLL_REGISTERS);
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
#ifdef _OPENMP
        uint8_t *mine = priv + (size_t)omp_get_thread_num() * ORC_HLL_REGISTERS;
#pragma omp for schedule(static)
#else
        uint8_t *mine = priv;
#endif
        for (uint64_t j = 0; j < n; j++) {
            uint8_t key[64];
            orc_gen_varlen_key(seed, start + j, key);
            long idx;
            int c = orc_hll_patlen(key, orc_gen_varlen_len(seed, start + j), &idx);
            if (c > mine[idx]) mine[idx] = (uint8_t)c;
        }
    }
    for (int t = 0; t < nthreads; t++)
        for (int j = 0; j < ORC_HLL_REGISTERS; j++)
            if (priv[(size_t)t * ORC_HLL_REGISTERS + j] > regs[j]) regs[j] = priv[(size_t)t * ORC_HLL_REGISTERS + j];
    free(priv);
}

void orc_gen_grouped(uint64_t seed, uint64_t G, uint64_t start, uint64_t n, uint32_t *groups, uint8_t *keys) {
    for (uint64_t j = 0; j < n; j++) {
        uint64_t i = start + j;
        groups[j] = (uint32_t)(orc_splitmix64(seed + 3 * i) % G);
        uint64_t lo = orc_splitmix64(seed + 3 * i + 1), hi = orc_splitmix64(seed + 3 * i + 2);
        memcpy(keys + 16 * j, &lo, 8);
        memcpy(keys + 16 * j + 8, &hi, 8);
    }
}

/* C5 Zipf(s) stress variant (restates rsk_gen.hip zipf_cdf / gen_grouped_zipf_kernel):
 * cdf[r] = floor(2^63 * sum_{q<=r+1} q^-s / sum_{q<=G} q^-s), cdf[G-1] = 2^63;
 * group of pair i = first r with (splitmix64(seed+3i) >> 1) < cdf[r]. */
void orc_zipf_cdf(uint64_t G, double s, uint64_t *cdf) {
    double total = 0.0, cum = 0.0;
    for (uint64_t r = 1; r <= G; r++) total += pow((double)r, -s);
    for (uint64_t r = 1; r <= G; r++) {
        cum += pow((double)r, -s);
        cdf[r - 1] = (uint64_t)ldexp(cum / total, 63);
    }
    cdf[G - 1] = 1ULL << 63;
}

static uint32_t zipf_rank(const uint64_t *cdf, uint64_t G, uint64_t u) {
    uint64_t lo = 0, hi = G - 1;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid;
        else lo = mid + 1;
    }
    return (uint32_t)lo;
}

void orc_gen_grouped_zipf(uint64_t seed, uint64_t G, double s, uint64_t start, uint64_t n, uint32_t *groups,
                          uint8_t *keys) {
    uint64_t *cdf = malloc(8 * G);
    orc_zipf_cdf(G, s, cdf);
    for (uint64_t j = 0; j < n; j++) {
        uint64_t i = start + j;
        groups[j] = zipf_rank(cdf, G, orc_splitmix64(seed + 3 * i) >> 1);
        uint64_t lo = orc_splitmix64(seed + 3 * i + 1), hi = orc_splitmix64(seed + 3 * i + 2);
        memcpy(keys + 16 * j, &lo, 8);
        memcpy(keys + 16 * j + 8, &hi, 8);
    }
    free(cdf);
}

/* Registers of the Zipf groups [0, gsub) (the hottest ones) over the whole
 * pair stream: regs is [gsub][16384].  Each of nthreads threads takes a
 * contiguous range of the pairs into private registers, max-merged at the end
 * (the hot groups get most pairs, so splitting by group would serialise). */
void orc_hll_add_gen_grouped_zipf_subset(uint8_t *regs, uint64_t G, uint64_t gsub, double s, uint64_t seed,
                                         uint64_t start, uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    uint64_t *cdf = malloc(8 * G);
    orc_zipf_cdf(G, s, cdf);
    const size_t per = (size_t)gsub * ORC_HLL_REGISTERS;
    uint8_t *priv = calloc((size_t)nthreads, per);
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
#ifdef _OPENMP
        const uint64_t t = (uint64_t)omp_get_thread_num(), nt = (uint64_t)omp_get_num_threads();
#else
        const uint64_t t = 0, nt = 1;
#endif
        uint8_t *mine = priv + t * per;
        for (uint64_t j = n * t / nt; j < n * (t + 1) / nt; j++) {
            const uint64_t i = start + j;
            const uint32_t g = zipf_rank(cdf, G, orc_splitmix64(seed + 3 * i) >> 1);
            if (g >= gsub) continue;
            uint8_t key[16];
            uint64_t lo = orc_splitmix64(seed + 3 * i + 1), hi = orc_splitmix64(seed + 3 * i + 2);
            memcpy(key, &lo, 8);
            memcpy(key + 8, &hi, 8);
            long idx;
            int c = orc_hll_patlen(key, 16, &idx);
            uint8_t *r = mine + (uint64_t)g * ORC_HLL_REGISTERS;
            if (c > r[idx]) r[idx] = (uint8_t)c;
        }
    }
    for (int t = 0; t < nthreads; t++)
        for (size_t j = 0; j < per; j++)
            if (priv[(size_t)t * per + j] > regs[j]) regs[j] = priv[(size_t)t * per + j];
    free(priv);
    free(cdf);
}

/* The groups of the uniform pair stream for pairs [start, start + n) (as
 * orc_gen_grouped, without the keys), on nthreads cores. */
void orc_gen_grouped_groups(uint64_t seed, uint64_t G, uint64_t start, uint64_t n, uint32_t *groups, int nthreads) {
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (uint64_t j = 0; j < n; j++) groups[j] = (uint32_t)(orc_splitmix64(seed + 3 * (start + j)) % G);
}

/* The groups of the Zipf pair stream for pairs [start, start + n) (as
 * orc_gen_grouped_zipf, without the keys), on nthreads cores. */
void orc_gen_grouped_zipf_groups(uint64_t seed, uint64_t G, double s, uint64_t start, uint64_t n, uint32_t *groups,
                                 int nthreads) {
    if (nthreads < 1) nthreads = 1;
    uint64_t *cdf = malloc(8 * G);
    orc_zipf_cdf(G, s, cdf);
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (uint64_t j = 0; j < n; j++) groups[j] = zipf_rank(cdf, G, orc_splitmix64(seed + 3 * (start + j)) >> 1);
    free(cdf);
}

/* A whole pool [G][16384] from pairs [start, start + n) whose groups are
 * given (groups[j]: ids >= G dropped) and whose keys are the grouped streams'
 * (splitmix64 of seed + 3i + 1, seed + 3i + 2): each of nthreads cores owns a
 * contiguous range of the groups and hashes only its pairs, so no two threads
 * write one row (a full-pool check of the grouped add, uniform or Zipf). */
void orc_hll_add_keys_by_groups(uint8_t *regs, uint64_t G, const uint32_t *groups, uint64_t seed, uint64_t start,
                                uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
#ifdef _OPENMP
        const uint64_t t = (uint64_t)omp_get_thread_num(), nt = (uint64_t)omp_get_num_threads();
#else
        const uint64_t t = 0, nt = 1;
#endif
        const uint64_t g0 = G * t / nt, g1 = G * (t + 1) / nt;
        for (uint64_t j = 0; j < n; j++) {
            const uint32_t g = groups[j];
            if (g < g0 || g >= g1) continue;
            const uint64_t i = start + j;
            uint8_t key[16];
            uint64_t lo = orc_splitmix64(seed + 3 * i + 1), hi = orc_splitmix64(seed + 3 * i + 2);
            memcpy(key, &lo, 8);
            memcpy(key + 8, &hi, 8);
            long idx;
            int c = orc_hll_patlen(key, 16, &idx);
            uint8_t *r = regs + (uint64_t)g * ORC_HLL_REGISTERS;
            if (c > r[idx]) r[idx] = (uint8_t)c;
        }
    }
}

/* Bloom query stream (C3): query q is an inserted key (index r>>1 mod n_ins
 * of the insert stream iseed) when r&1, else a fresh key. */
void orc_gen_queries16(uint64_t qseed, uint64_t iseed, uint64_t n_ins, uint64_t start, uint64_t n, uint8_t *out) {
    for (uint64_t j = 0; j < n; j++) {
        uint64_t q = start + j;
        uint64_t r = orc_splitmix64(qseed + 3 * q);
        uint64_t lo, hi;
        if (r & 1) {
            uint64_t i = (r >> 1) % n_ins;
            lo = orc_splitmix64(iseed + 2 * i);
            hi = orc_splitmix64(iseed + 2 * i + 1);
        } else {
            /* bit 63 set: never a state of the insert stream (iseed + j, j < 2^62) */
            lo = orc_splitmix64((qseed + 3 * q + 1) | 0x8000000000000000ULL);
            hi = orc_splitmix64((qseed + 3 * q + 2) | 0x8000000000000000ULL);
        }
        memcpy(out + 16 * j, &lo, 8);
        memcpy(out + 16 * j + 8, &hi, 8);
    }
}

void orc_hll_add_gen16(uint8_t *regs, uint64_t seed, uint64_t start, uint64_t n, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 1) {
        uint8_t *priv = (uint8_t *)calloc((size_t)nthreads, ORC_HLL_REGISTERS);
#pragma omp parallel num_threads(nthreads)
        {
            int t = omp_get_thread_num();
            uint8_t *mine = priv + (size_t)t * ORC_HLL_REGISTERS;
#pragma omp for schedule(static)
            for (uint64_t j = 0; j < n; j++) {
                uint64_t i = start + j;
                uint8_t key[16];
                uint64_t lo = orc_splitmix64(seed + 2 * i), hi = orc_splitmix64(seed + 2 * i + 1);
                memcpy(key, &lo, 8);
                memcpy(key + 8, &hi, 8);
                long idx;
                int c = orc_hll_patlen(key, 16, &idx);
                if (c > mine[idx]) mine[idx] = (uint8_t)c;
            }
        }
        for (int t = 0; t < nthreads; t++)
            for (int j = 0; j < ORC_HLL_REGISTERS; j++)
                if (priv[(size_t)t * ORC_HLL_REGISTERS + j] > regs[j]) regs[j] = priv[(size_t)t * ORC_HLL_REGISTERS + j];
        free(priv);
        return;
    }
#endif
    (void)nthreads;
    for (uint64_t j = 0; j < n; j++) {
        uint64_t i = start + j;
        uint8_t key[16];
        uint64_t lo = orc_splitmix64(seed + 2 * i), hi = orc_splitmix64(seed + 2 * i + 1);
        memcpy(key, &lo, 8);
        memcpy(key + 8, &hi, 8);
        long idx;
        int c = orc_hll_patlen(key, 16, &idx);
        if (c > regs[idx]) regs[idx] = (uint8_t)c;
    }
}

void orc_hll_add_gen_grouped(uint8_t *regs, uint64_t G, uint64_t seed, uint64_t start, uint64_t n) {
    for (uint64_t j = 0; j < n; j++) {
        uint32_t g;
        uint8_t key[16];
        orc_gen_grouped(seed, G, start + j, 1, &g, key);
        long idx;
        int c = orc_hll_patlen(key, 16, &idx);
        uint8_t *r = regs + (uint64_t)g * ORC_HLL_REGISTERS;
        if (c > r[idx]) r[idx] = (uint8_t)c;
    }
}

/* The same restricted to groups [0, gsub): regs is [gsub][16384]; only the
 * pairs of those groups are hashed (a full-size check of a group sample),
 * on nthreads cores, each thread owning a contiguous range of the groups. */
void orc_hll_add_gen_grouped_subset(uint8_t *regs, uint64_t G, uint64_t gsub, uint64_t seed, uint64_t start,
                                    uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
#ifdef _OPENMP
        const uint64_t t = (uint64_t)omp_get_thread_num(), nt = (uint64_t)omp_get_num_threads();
#else
        const uint64_t t = 0, nt = 1;
#endif
        const uint64_t g0 = gsub * t / nt, g1 = gsub * (t + 1) / nt;
        for (uint64_t j = 0; j < n; j++) {
            const uint64_t i = start + j;
            const uint32_t g = (uint32_t)(orc_splitmix64(seed + 3 * i) % G);
            if (g < g0 || g >= g1) continue;
            uint8_t key[16];
            uint64_t lo = orc_splitmix64(seed + 3 * i + 1), hi = orc_splitmix64(seed + 3 * i + 2);
            memcpy(key, &lo, 8);
            memcpy(key + 8, &hi, 8);
            long idx;
            int c = orc_hll_patlen(key, 16, &idx);
            uint8_t *r = regs + (uint64_t)g * ORC_HLL_REGISTERS;
            if (c > r[idx]) r[idx] = (uint8_t)c;
        }
    }
}

/* Any set of groups: ids[0..nids) (distinct, < G); regs is [nids][16384],
 * row s = group ids[s].  Each thread owns the rows s with s % nt == t. */
void orc_hll_add_gen_grouped_ids(uint8_t *regs, uint64_t G, const uint64_t *ids, uint64_t nids, uint64_t seed,
                                 uint64_t start, uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    uint32_t *slot = malloc(sizeof(uint32_t) * (size_t)G);
    if (!slot) return;
    for (uint64_t g = 0; g < G; ++g) slot[g] = UINT32_MAX;
    for (uint64_t s = 0; s < nids; ++s) slot[ids[s]] = (uint32_t)s;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
#ifdef _OPENMP
        const uint32_t t = (uint32_t)omp_get_thread_num(), nt = (uint32_t)omp_get_num_threads();
#else
        const uint32_t t = 0, nt = 1;
#endif
        for (uint64_t j = 0; j < n; j++) {
            const uint64_t i = start + j;
            const uint32_t s = slot[orc_splitmix64(seed + 3 * i) % G];
            if (s == UINT32_MAX || s % nt != t) continue;
            uint8_t key[16];
            uint64_t lo = orc_splitmix64(seed + 3 * i + 1), hi = orc_splitmix64(seed + 3 * i + 2);
            memcpy(key, &lo, 8);
            memcpy(key + 8, &hi, 8);
            long idx;
            int c = orc_hll_patlen(key, 16, &idx);
            uint8_t *r = regs + (uint64_t)s * ORC_HLL_REGISTERS;
            if (c > r[idx]) r[idx] = (uint8_t)c;
        }
    }
    free(slot);
}

/* ===================================================================== */
/* Redis 3.2.0 dense register access (HLL_DENSE_GET/SET_REGISTER).        */
/* ===================================================================== */
int orc_hll_dense_get(const uint8_t *p, int j) {
    unsigned long byte = (unsigned long)j * ORC_HLL_BITS / 8;
    unsigned long fb = (unsigned long)j * ORC_HLL_BITS & 7;
    unsigned long fb8 = 8 - fb;
    unsigned long b0 = p[byte];
    unsigned long b1 = (byte + 1 < (ORC_HLL_REGISTERS * ORC_HLL_BITS + 7) / 8) ? p[byte + 1] : 0;
    return (int)(((b0 >> fb) | (b1 << fb8)) & 63);
}

void orc_hll_dense_set(uint8_t *p, int j, int v) {
    unsigned long byte = (unsigned long)j * ORC_HLL_BITS / 8;
    unsigned long fb = (unsigned long)j * ORC_HLL_BITS & 7;
    unsigned long fb8 = 8 - fb;
    unsigned long val = (unsigned long)v;
    p[byte] &= (uint8_t)~(63UL << fb);
    p[byte] |= (uint8_t)(val << fb);
    if (byte + 1 < (ORC_HLL_REGISTERS * ORC_HLL_BITS + 7) / 8) {
        p[byte + 1] &= (uint8_t)~(63UL >> fb8);
        p[byte + 1] |= (uint8_t)(val >> fb8);
    }
}

static double PE[64];
static int pe_init = 0;
static void init_pe(void) {
    if (pe_init) return;
    PE[0] = 1;
    for (int j = 1; j < 64; j++) PE[j] = 1.0 / (double)(1ULL << j);
    pe_init = 1;
}

/* hllDenseSum: 1024 groups of 16 registers, each group summed as
 * (PE0+PE1)+(PE2+PE3)+...+(PE14+PE15), left to right, then E += group. */
double orc_hll_dense_sum(const uint8_t *registers, int *ezp) {
    init_pe();
    double E = 0;
    int ez = 0;
    for (int g = 0; g < ORC_HLL_REGISTERS / 16; g++) {
        int r[16];
        for (int t = 0; t < 16; t++) {
            r[t] = orc_hll_dense_get(registers, g * 16 + t);
            if (r[t] == 0) ez++;
        }
        E += (PE[r[0]] + PE[r[1]]) + (PE[r[2]] + PE[r[3]]) + (PE[r[4]] + PE[r[5]]) +
             (PE[r[6]] + PE[r[7]]) + (PE[r[8]] + PE[r[9]]) + (PE[r[10]] + PE[r[11]]) +
             (PE[r[12]] + PE[r[13]]) + (PE[r[14]] + PE[r[15]]);
    }
    *ezp = ez;
    return E;
}

/* hllRawSum: 8 registers per u64 word; all-zero words add 8 to ez; zeros
 * are added once at the end (E += ez). */
double orc_hll_raw_sum(const uint8_t *registers, int *ezp) {
    init_pe();
    double E = 0;
    int ez = 0;
    for (int j = 0; j < ORC_HLL_REGISTERS / 8; j++) {
        const uint8_t *b = registers + 8 * j;
        if (ld64(b) == 0) {
            ez += 8;
        } else {
            for (int t = 0; t < 8; t++) {
                if (b[t]) E += PE[b[t]];
                else ez++;
            }
        }
    }
    E += ez;
    *ezp = ez;
    return E;
}

#define SP_IS_ZERO(p) (((*(p)) & 0xc0) == 0)
#define SP_IS_XZERO(p) (((*(p)) & 0xc0) == 0x40)
#define SP_ZERO_LEN(p) (((*(p)) & 0x3f) + 1)
#define SP_XZERO_LEN(p) (((((*(p)) & 0x3f) << 8) | (*((p) + 1))) + 1)
#define SP_VAL_VALUE(p) ((((*(p)) >> 2) & 0x1f) + 1)
#define SP_VAL_LEN(p) (((*(p)) & 0x3) + 1)

/* hllSparseSum: VAL runs add PE[v]*runlen in stream order, zeros at the end. */
double orc_hll_sparse_sum(const uint8_t *sparse, int sparselen, int *ezp, int *invalid) {
    init_pe();
    double E = 0;
    int ez = 0, idx = 0, runlen, regval;
    const uint8_t *end = sparse + sparselen, *p = sparse;
    while (p < end) {
        if (SP_IS_ZERO(p)) {
            runlen = SP_ZERO_LEN(p);
            idx += runlen;
            ez += runlen;
            p++;
        } else if (SP_IS_XZERO(p)) {
            runlen = SP_XZERO_LEN(p);
            idx += runlen;
            ez += runlen;
            p += 2;
        } else {
            runlen = SP_VAL_LEN(p);
            regval = SP_VAL_VALUE(p);
            idx += runlen;
            E += PE[regval] * runlen;
            p++;
        }
    }
    if (idx != ORC_HLL_REGISTERS && invalid) *invalid = 1;
    E += ez;
    *ezp = ez;
    return E;
}

/* hllCount tail (Redis 3.2.0): raw estimate, linear counting below 2.5m,
 * polynomial bias correction below 72000. */
uint64_t orc_hll_estimate(double E, int ez) {
    double m = ORC_HLL_REGISTERS;
    double alpha = 0.7213 / (1 + 1.079 / m);
    E = (1 / E) * alpha * m * m;
    if (E < m * 2.5 && ez != 0) {
        E = m * log(m / ez);
    } else if (m == 16384 && E < 72000) {
        double bias = 5.9119 * 1.0e-18 * (E * E * E * E)
                      - 1.4253 * 1.0e-12 * (E * E * E) +
                      1.2940 * 1.0e-7 * (E * E)
                      - 5.2921 * 1.0e-3 * E +
                      83.3216;
        E -= E * (bias / 100);
    }
    return (uint64_t)E;
}

uint64_t orc_hll_count_raw(const uint8_t *raw) {
    int ez;
    double E = orc_hll_raw_sum(raw, &ez);
    return orc_hll_estimate(E, ez);
}

uint64_t orc_hll_count_dense_regs(const uint8_t *raw) {
    uint8_t dense[ORC_HLL_DENSE_SIZE - ORC_HLL_HDR_SIZE];
    memset(dense, 0, sizeof dense);
    for (int j = 0; j < ORC_HLL_REGISTERS; j++) orc_hll_dense_set(dense, j, raw[j]);
    int ez;
    double E = orc_hll_dense_sum(dense, &ez);
    return orc_hll_estimate(E, ez);
}

/* ===================================================================== */
/* Redis HLL string encodings.                                             */
/* ===================================================================== */
static void put_hdr(uint8_t *out, int encoding, const uint8_t card[8]) {
    out[0] = 'H'; out[1] = 'Y'; out[2] = 'L'; out[3] = 'L';
    out[4] = (uint8_t)encoding;
    out[5] = out[6] = out[7] = 0;
    if (card) memcpy(out + 8, card, 8);
    else memset(out + 8, 0, 8);
}

int orc_hll_encode_dense(const uint8_t *raw, const uint8_t card[8], uint8_t *out, size_t cap) {
    if (cap < ORC_HLL_DENSE_SIZE) return -1;
    memset(out, 0, ORC_HLL_DENSE_SIZE);
    put_hdr(out, 0, card);
    for (int j = 0; j < ORC_HLL_REGISTERS; j++) {
        if (raw[j] > 63) return -1;
        orc_hll_dense_set(out + ORC_HLL_HDR_SIZE, j, raw[j]);
    }
    return ORC_HLL_DENSE_SIZE;
}

/* Canonical sparse encoding: zero runs as XZERO (>64) / ZERO, value runs as
 * VAL opcodes of at most 4.  Returns -1 when a register exceeds 32 (the
 * sparse form cannot hold it; Redis promotes to dense). */
int orc_hll_encode_sparse(const uint8_t *raw, const uint8_t card[8], uint8_t *out, size_t cap) {
    size_t o = ORC_HLL_HDR_SIZE;
    if (cap < ORC_HLL_HDR_SIZE) return -1;
    put_hdr(out, 1, card);
    int j = 0;
    while (j < ORC_HLL_REGISTERS) {
        int v = raw[j], run = 1;
        while (j + run < ORC_HLL_REGISTERS && raw[j + run] == v) run++;
        if (v == 0) {
            int left = run;
            while (left > 0) {
                if (left > 64) {
                    int l = left > 16384 ? 16384 : left;
                    if (o + 2 > cap) return -1;
                    out[o++] = (uint8_t)(((l - 1) >> 8) | 0x40);
                    out[o++] = (uint8_t)((l - 1) & 0xff);
                    left -= l;
                } else {
                    if (o + 1 > cap) return -1;
                    out[o++] = (uint8_t)(left - 1);
                    left = 0;
                }
            }
        } else {
            if (v > 32) return -1;
            int left = run;
            while (left > 0) {
                int l = left > 4 ? 4 : left;
                if (o + 1 > cap) return -1;
                out[o++] = (uint8_t)((((v - 1) << 2) | (l - 1)) | 0x80);
                left -= l;
            }
        }
        j += run;
    }
    return (int)o;
}

/* isHLLObjectOrReply + hllMerge-style decode into raw registers.
 * Returns 0 ok, -1 WRONGTYPE (not a valid HLL string), -2 INVALIDOBJ
 * (corrupted sparse payload). */
int orc_hll_decode(const uint8_t *buf, size_t len, uint8_t *raw, int *encoding) {
    if (len < ORC_HLL_HDR_SIZE) return -1;
    if (buf[0] != 'H' || buf[1] != 'Y' || buf[2] != 'L' || buf[3] != 'L') return -1;
    if (buf[4] > 1) return -1;
    if (buf[4] == 0 && len != ORC_HLL_DENSE_SIZE) return -1;
    if (encoding) *encoding = buf[4];
    memset(raw, 0, ORC_HLL_REGISTERS);
    if (buf[4] == 0) {
        for (int j = 0; j < ORC_HLL_REGISTERS; j++) raw[j] = (uint8_t)orc_hll_dense_get(buf + ORC_HLL_HDR_SIZE, j);
        return 0;
    }
    const uint8_t *p = buf + ORC_HLL_HDR_SIZE, *end = buf + len;
    long i = 0;
    while (p < end) {
        long runlen;
        if (SP_IS_ZERO(p)) {
            runlen = SP_ZERO_LEN(p);
            i += runlen;
            p++;
        } else if (SP_IS_XZERO(p)) {
            runlen = SP_XZERO_LEN(p);
            i += runlen;
            p += 2;
        } else {
            runlen = SP_VAL_LEN(p);
            int regval = SP_VAL_VALUE(p);
            if ((runlen + i) > ORC_HLL_REGISTERS) break; /* overflow */
            while (runlen--) {
                if (regval > raw[i]) raw[i] = (uint8_t)regval;
                i++;
            }
            p++;
        }
    }
    if (i != ORC_HLL_REGISTERS) return -2;
    return 0;
}

/* PFCOUNT on a single stored key: cached value when card[7] bit 7 is clear,
 * else hllCount in the key's own encoding order. */
int orc_hll_count_string(const uint8_t *buf, size_t len, uint64_t *out) {
    uint8_t raw[ORC_HLL_REGISTERS];
    int enc;
    int rc = orc_hll_decode(buf, len, raw, &enc);
    if (rc) return rc;
    const uint8_t *card = buf + 8;
    if ((card[7] & 0x80) == 0) {
        uint64_t c = 0;
        for (int t = 0; t < 8; t++) c |= (uint64_t)card[t] << (8 * t);
        *out = c;
        return 0;
    }
    int ez, invalid = 0;
    double E;
    if (enc == 0) E = orc_hll_dense_sum(buf + ORC_HLL_HDR_SIZE, &ez);
    else E = orc_hll_sparse_sum(buf + ORC_HLL_HDR_SIZE, (int)(len - ORC_HLL_HDR_SIZE), &ez, &invalid);
    if (invalid) return -2;
    *out = orc_hll_estimate(E, ez);
    return 0;
}

/* ===================================================================== */
/* XXH64 (OpenHFT LongHashFunction.xx_r39(), seed 0).                      */
/* ===================================================================== */
#define XP1 0x9E3779B185EBCA87ULL
#define XP2 0xC2B2AE3D27D4EB4FULL
#define XP3 0x165667B19E3779F9ULL
#define XP4 0x85EBCA77C2B2AE63ULL
#define XP5 0x27D4EB2F165667C5ULL
static inline uint64_t xround(uint64_t acc, uint64_t in) {
    acc += in * XP2;
    acc = rotl64(acc, 31);
    return acc * XP1;
}
static inline uint64_t xmerge(uint64_t acc, uint64_t val) {
    acc ^= xround(0, val);
    return acc * XP1 + XP4;
}
uint64_t orc_xxh64(const void *key, size_t len, uint64_t seed) {
    const uint8_t *p = (const uint8_t *)key, *end = p + len;
    uint64_t h;
    if (len >= 32) {
        const uint8_t *limit = end - 32;
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        do {
            v1 = xround(v1, ld64(p));
            v2 = xround(v2, ld64(p + 8));
            v3 = xround(v3, ld64(p + 16));
            v4 = xround(v4, ld64(p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) {
        h ^= xround(0, ld64(p));
        h = rotl64(h, 27) * XP1 + XP4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)ld32(p) * XP1;
        h = rotl64(h, 23) * XP2 + XP3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * XP5;
        h = rotl64(h, 11) * XP1;
        p++;
    }
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

/* ===================================================================== */
/* farmhash 1.1: farmhashna::Hash64 and farmhashuo::Hash64                 */
/* (OpenHFT LongHashFunction.farmUo()).                                    */
/* ===================================================================== */
static const uint64_t k0 = 0xc3a5c85c97cb3127ULL;
static const uint64_t k1 = 0xb492b66fbe98f273ULL;
static const uint64_t k2 = 0x9ae16a3b2f90404fULL;

static inline uint64_t shift_mix(uint64_t v) { return v ^ (v >> 47); }
static inline uint64_t hash_len16(uint64_t u, uint64_t v, uint64_t mul) {
    uint64_t a = (u ^ v) * mul;
    a ^= (a >> 47);
    uint64_t b = (v ^ a) * mul;
    b ^= (b >> 47);
    b *= mul;
    return b;
}
static uint64_t na_len0to16(const uint8_t *s, size_t len) {
    if (len >= 8) {
        uint64_t mul = k2 + len * 2;
        uint64_t a = ld64(s) + k2;
        uint64_t b = ld64(s + len - 8);
        uint64_t c = rotr64(b, 37) * mul + a;
        uint64_t d = (rotr64(a, 25) + b) * mul;
        return hash_len16(c, d, mul);
    }
    if (len >= 4) {
        uint64_t mul = k2 + len * 2;
        uint64_t a = ld32(s);
        return hash_len16(len + (a << 3), ld32(s + len - 4), mul);
    }
    if (len > 0) {
        uint8_t a = s[0], b = s[len >> 1], c = s[len - 1];
        uint32_t y = (uint32_t)a + ((uint32_t)b << 8);
        uint32_t z = (uint32_t)len + ((uint32_t)c << 2);
        return shift_mix((uint64_t)y * k2 ^ (uint64_t)z * k0) * k2;
    }
    return k2;
}
static uint64_t na_len17to32(const uint8_t *s, size_t len) {
    uint64_t mul = k2 + len * 2;
    uint64_t a = ld64(s) * k1;
    uint64_t b = ld64(s + 8);
    uint64_t c = ld64(s + len - 8) * mul;
    uint64_t d = ld64(s + len - 16) * k2;
    return hash_len16(rotr64(a + b, 43) + rotr64(c, 30) + d, a + rotr64(b + k2, 18) + c, mul);
}
static uint64_t na_len33to64(const uint8_t *s, size_t len) {
    uint64_t mul = k2 + len * 2;
    uint64_t a = ld64(s) * k2;
    uint64_t b = ld64(s + 8);
    uint64_t c = ld64(s + len - 8) * mul;
    uint64_t d = ld64(s + len - 16) * k2;
    uint64_t y = rotr64(a + b, 43) + rotr64(c, 30) + d;
    uint64_t z = hash_len16(y, a + rotr64(b + k2, 18) + c, mul);
    uint64_t e = ld64(s + 16) * mul;
    uint64_t f = ld64(s + 24);
    uint64_t g = (y + ld64(s + len - 32)) * mul;
    uint64_t h = (z + ld64(s + len - 24)) * mul;
    return hash_len16(rotr64(e + f, 43) + rotr64(g, 30) + h, e + rotr64(f + a, 18) + g, mul);
}
typedef struct { uint64_t first, second; } u64pair;
static inline u64pair weak32(uint64_t w, uint64_t x, uint64_t y, uint64_t z, uint64_t a, uint64_t b) {
    a += w;
    b = rotr64(b + a + z, 21);
    uint64_t c = a;
    a += x;
    a += y;
    b += rotr64(a, 44);
    u64pair r = {a + z, b + c};
    return r;
}
static inline u64pair weak32s(const uint8_t *s, uint64_t a, uint64_t b) {
    return weak32(ld64(s), ld64(s + 8), ld64(s + 16), ld64(s + 24), a, b);
}

uint64_t orc_farmhash_na64(const void *key, size_t len) {
    const uint8_t *s = (const uint8_t *)key;
    const uint64_t seed = 81;
    if (len <= 32) {
        if (len <= 16) return na_len0to16(s, len);
        return na_len17to32(s, len);
    } else if (len <= 64) {
        return na_len33to64(s, len);
    }
    uint64_t x = seed;
    uint64_t y = seed * k1 + 113;
    uint64_t z = shift_mix(y * k2 + 113) * k2;
    u64pair v = {0, 0}, w = {0, 0};
    x = x * k2 + ld64(s);
    const uint8_t *end = s + ((len - 1) / 64) * 64;
    const uint8_t *last64 = end + ((len - 1) & 63) - 63;
    do {
        x = rotr64(x + y + v.first + ld64(s + 8), 37) * k1;
        y = rotr64(y + v.second + ld64(s + 48), 42) * k1;
        x ^= w.second;
        y += v.first + ld64(s + 40);
        z = rotr64(z + w.first, 33) * k1;
        v = weak32s(s, v.second * k1, x + w.first);
        w = weak32s(s + 32, z + w.second, y + ld64(s + 16));
        uint64_t t = z; z = x; x = t;
        s += 64;
    } while (s != end);
    uint64_t mul = k1 + ((z & 0xff) << 1);
    s = last64;
    w.first += ((len - 1) & 63);
    v.first += w.first;
    w.first += v.first;
    x = rotr64(x + y + v.first + ld64(s + 8), 37) * mul;
    y = rotr64(y + v.second + ld64(s + 48), 42) * mul;
    x ^= w.second * 9;
    y += v.first * 9 + ld64(s + 40);
    z = rotr64(z + w.first, 33) * mul;
    v = weak32s(s, v.second * mul, x + w.first);
    w = weak32s(s + 32, z + w.second, y + ld64(s + 16));
    { uint64_t t = z; z = x; x = t; }
    return hash_len16(hash_len16(v.first, w.first, mul) + shift_mix(y) * k0 + z,
                      hash_len16(v.second, w.second, mul) + x, mul);
}

static inline uint64_t uo_h(uint64_t x, uint64_t y, uint64_t mul, int r) {
    uint64_t a = (x ^ y) * mul;
    a ^= (a >> 47);
    uint64_t b = (y ^ a) * mul;
    return rotr64(b, r) * mul;
}

/* farmhashuo::Hash64WithSeeds(s, len, 81, 0) for len > 64.  PARITY UNPINNED:
 * no oracle or golden vector for this path exists in the container. */
static uint64_t uo_seeds(const uint8_t *s, size_t len, uint64_t seed0, uint64_t seed1) {
    uint64_t x = seed0;
    uint64_t y = seed1 * k2 + 113;
    uint64_t z = shift_mix(y * k2) * k2;
    u64pair v = {seed0, seed1}, w = {0, 0};
    uint64_t u = x - z;
    x *= k2;
    uint64_t mul = k2 + (u & 0x82);
    const uint8_t *end = s + ((len - 1) / 64) * 64;
    const uint8_t *last64 = end + ((len - 1) & 63) - 63;
    do {
        uint64_t a0 = ld64(s), a1 = ld64(s + 8), a2 = ld64(s + 16), a3 = ld64(s + 24);
        uint64_t a4 = ld64(s + 32), a5 = ld64(s + 40), a6 = ld64(s + 48), a7 = ld64(s + 56);
        x += a0 + a1;
        y += a2;
        z += a3;
        v.first += a4;
        v.second += a5 + a1;
        w.first += a6;
        w.second += a7;

        x = rotr64(x, 26);
        x *= 9;
        y = rotr64(y, 29);
        z *= mul;
        v.first = rotr64(v.first, 33);
        v.second = rotr64(v.second, 30);
        w.first ^= x;
        w.first *= 9;
        z = rotr64(z, 32);
        z += w.second;
        w.second += z;
        z *= 9;
        { uint64_t t = u; u = y; y = t; }

        z += a0 + a6;
        v.first += a2;
        v.second += a3;
        w.first += a4;
        w.second += a5 + a6;
        x += a1;
        y += a7;

        y += v.first;
        v.first += x - y;
        v.second += w.first;
        w.first += v.second;
        w.second += x - y;
        x += w.second;
        w.second = rotr64(w.second, 34);
        { uint64_t t = u; u = z; z = t; }
        s += 64;
    } while (s != end);
    s = last64;
    u *= 9;
    v.second = rotr64(v.second, 28);
    v.first = rotr64(v.first, 20);
    w.first += ((len - 1) & 63);
    u += y;
    y += u;
    x = rotr64(y - x + v.first + ld64(s + 8), 37) * mul;
    y = rotr64(y ^ v.second ^ ld64(s + 48), 42) * mul;
    x ^= w.second * 9;
    y += v.first + ld64(s + 40);
    z = rotr64(z + w.first, 33) * mul;
    v = weak32s(s, v.second * mul, x + w.first);
    w = weak32s(s + 32, z + w.second, y + ld64(s + 16));
    return uo_h(hash_len16(v.first + x, w.first ^ y, mul) + z - u,
                uo_h(v.second + w.second, w.first + v.first, mul, 30) + x, mul, 31);
}

uint64_t orc_farmhash_uo64(const void *key, size_t len) {
    if (len <= 64) return orc_farmhash_na64(key, len);
    return uo_seeds((const uint8_t *)key, len, 81, 0);
}

/* ===================================================================== */
/* RedissonBloomFilter.java arithmetic.                                    */
/* ===================================================================== */
/* Java (long) cast of a double: NaN -> 0, saturating, truncating. */
static int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}
static int32_t java_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}
/* Math.round(double) (Java 6-8: floor(a + 0.5) except the 0.49999999999999994 case). */
static int64_t java_round(double a) {
    if (a == 0x1.fffffffffffffp-2) return 0;
    return java_d2l(floor(a + 0.5));
}

/* optimalNumOfBits, RedissonBloomFilter.java:73-78. */
int64_t orc_bloom_optimal_bits(int64_t n, double p) {
    if (p == 0) p = 4.9e-324; /* Double.MIN_VALUE */
    return java_d2l((double)(-n) * log(p) / (log(2) * log(2)));
}

/* optimalNumOfHashFunctions, RedissonBloomFilter.java:69-71. */
int32_t orc_bloom_optimal_k(int64_t n, int64_t m) {
    int32_t r = (int32_t)java_round((double)m / (double)n * log(2));
    return r > 1 ? r : 1;
}

/* hash(), RedissonBloomFilter.java:116-131. */
void orc_bloom_indexes(const uint8_t *key, size_t len, int k, int64_t size, int64_t *out) {
    uint64_t h1 = orc_xxh64(key, len, 0);
    uint64_t h2 = orc_farmhash_uo64(key, len);
    uint64_t h = h1;
    for (int i = 0; i < k; i++) {
        out[i] = (int64_t)((h & 0x7FFFFFFFFFFFFFFFULL) % (uint64_t)size);
        if (i % 2 == 0) h += h2;
        else h += h1;
    }
}

/* count(), RedissonBloomFilter.java:198. */
int32_t orc_bloom_count(int64_t size, int k, int64_t bitcount) {
    return java_d2i((double)(-size) / ((double)k) * log(1 - (double)bitcount / ((double)size)));
}

/* Redis bitops.c SETBIT/GETBIT: byte = off>>3, bit = 7 - (off&7). */
int orc_setbit(uint8_t *bits, uint64_t off, int v) {
    uint64_t byte = off >> 3;
    int bit = 7 - (int)(off & 7);
    int old = (bits[byte] >> bit) & 1;
    bits[byte] &= (uint8_t)~(1 << bit);
    bits[byte] |= (uint8_t)((v & 1) << bit);
    return old;
}
int orc_getbit(const uint8_t *bits, uint64_t off) {
    return (bits[off >> 3] >> (7 - (int)(off & 7))) & 1;
}
uint64_t orc_bitcount(const uint8_t *bits, uint64_t nbytes) {
    uint64_t c = 0;
    for (uint64_t i = 0; i < nbytes; i++) c += (uint64_t)__builtin_popcount(bits[i]);
    return c;
}

/* add(), RedissonBloomFilter.java:80-114: k SETBITs; the result is true iff
 * one of setbit_0..setbit_{k-2} found the bit clear (subList(1,size-1)). */
void orc_bloom_add_batch(uint8_t *bits, int64_t size, int k, const uint8_t *data,
                         const uint64_t *offsets, uint32_t fixed_len, uint64_t n, uint8_t *added_out) {
    int64_t idx[64];
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p = offsets ? data + offsets[i] : data + i * (uint64_t)fixed_len;
        size_t len = offsets ? (size_t)(offsets[i + 1] - offsets[i]) : fixed_len;
        orc_bloom_indexes(p, len, k, size, idx);
        int added = 0;
        for (int t = 0; t < k; t++) {
            int old = orc_setbit(bits, (uint64_t)idx[t], 1);
            if (t < k - 1 && old == 0) added = 1;
        }
        if (added_out) added_out[i] = (uint8_t)added;
    }
}

/* The C3 insert stream (gen_keys16 keys start..start+n-1) on nthreads cores:
 * SETBIT of all k indices by relaxed atomic byte OR (bits are only set, so
 * the final string is order-independent).  k <= 64. */
void orc_bloom_add_gen16_mt(uint8_t *bits, int64_t size, int k, uint64_t seed, uint64_t start, uint64_t n,
                            int nthreads) {
    if (k > 64) return;
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
#endif
    for (uint64_t j = 0; j < n; j++) {
        uint8_t key[16];
        uint64_t i = start + j, lo = orc_splitmix64(seed + 2 * i), hi = orc_splitmix64(seed + 2 * i + 1);
        memcpy(key, &lo, 8);
        memcpy(key + 8, &hi, 8);
        int64_t idx[64];
        orc_bloom_indexes(key, 16, k, size, idx);
        for (int t = 0; t < k; t++)
            __atomic_fetch_or(&bits[(uint64_t)idx[t] >> 3], (uint8_t)(0x80u >> (idx[t] & 7)), __ATOMIC_RELAXED);
    }
    (void)nthreads;
}

/* contains() over the C3 query stream (orc_gen_queries16) on nthreads cores;
 * replies into out (may be NULL), returns the number of true replies. */
uint64_t orc_bloom_contains_gen_queries_mt(const uint8_t *bits, int64_t size, int k, uint64_t qseed, uint64_t iseed,
                                           uint64_t n_ins, uint64_t start, uint64_t n, uint8_t *out, int nthreads) {
    uint64_t trues = 0;
    if (k > 64) return 0;
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static) reduction(+ : trues)
#endif
    for (uint64_t j = 0; j < n; j++) {
        uint8_t key[16];
        orc_gen_queries16(qseed, iseed, n_ins, start + j, 1, key);
        int64_t idx[64];
        orc_bloom_indexes(key, 16, k, size, idx);
        int r = 1;
        for (int t = 0; t < k - 1; t++)
            if (!orc_getbit(bits, (uint64_t)idx[t])) { r = 0; break; }
        if (out) out[j] = (uint8_t)r;
        trues += (uint64_t)r;
    }
    (void)nthreads;
    return trues;
}

/* add() replies of sampled keys of the C3 insert stream (gen_keys16 keys
 * 0..n-1 added in ONE batch to an empty filter), on nthreads cores.  Key i
 * answers true iff one of its probes t < k-1 is the first SETBIT of its bit in
 * sequence order p = i k + t (the bit was clear before the batch), so only the
 * minimum p over the probes of the sample's bits is needed: those bits go in
 * a hash table (min p, atomically lowered by every probe of the stream that
 * hits one; a small bitmap screens the rest).  sample[] ascending, k <= 64. */
void orc_bloom_add_replies_sample_gen16_mt(int64_t size, int k, uint64_t seed, uint64_t n, const uint64_t *sample,
                                           uint64_t ns, uint8_t *out, int nthreads) {
    if (k > 64 || k < 1) return;
    const uint64_t EMPTY = ~0ull;
    uint64_t want = 4 * ns * (uint64_t)(k > 1 ? k - 1 : 1) + 16, cap = 16;
    int lg = 4;
    while (cap < want) { cap <<= 1; lg++; }
    uint64_t *tbit = (uint64_t *)malloc(cap * 8), *tmin = (uint64_t *)malloc(cap * 8);
    const int SCR = 27;
    uint64_t *scr = (uint64_t *)calloc((1ull << SCR) / 64, 8);
    for (uint64_t e = 0; e < cap; e++) { tbit[e] = EMPTY; tmin[e] = EMPTY; }
    int64_t *sidx = (int64_t *)malloc(ns * 64 * 8);
    for (uint64_t j = 0; j < ns; j++) {
        uint8_t key[16];
        orc_gen_keys16(seed, sample[j], 1, key);
        orc_bloom_indexes(key, 16, k, size, sidx + j * 64);
        for (int t = 0; t < k - 1; t++) {
            const uint64_t b = (uint64_t)sidx[j * 64 + t];
            uint64_t e = (b * 0x9E3779B97F4A7C15ull) >> (64 - lg);
            while (tbit[e] != EMPTY && tbit[e] != b) e = (e + 1) & (cap - 1);
            tbit[e] = b;
            const uint64_t h = (b * 0xD6E8FEB86659FD93ull) >> (64 - SCR);
            scr[h >> 6] |= 1ull << (h & 63);
        }
    }
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
#endif
    for (uint64_t i = 0; i < n; i++) {
        uint8_t key[16];
        uint64_t lo = orc_splitmix64(seed + 2 * i), hi = orc_splitmix64(seed + 2 * i + 1);
        memcpy(key, &lo, 8);
        memcpy(key + 8, &hi, 8);
        int64_t idx[64];
        orc_bloom_indexes(key, 16, k, size, idx);
        for (int t = 0; t < k; t++) {
            const uint64_t b = (uint64_t)idx[t];
            const uint64_t h = (b * 0xD6E8FEB86659FD93ull) >> (64 - SCR);
            if (!((scr[h >> 6] >> (h & 63)) & 1)) continue;
            uint64_t e = (b * 0x9E3779B97F4A7C15ull) >> (64 - lg);
            while (tbit[e] != EMPTY && tbit[e] != b) e = (e + 1) & (cap - 1);
            if (tbit[e] != b) continue;
            const uint64_t p = i * (uint64_t)k + (uint64_t)t;
            uint64_t cur = __atomic_load_n(&tmin[e], __ATOMIC_RELAXED);
            while (p < cur && !__atomic_compare_exchange_n(&tmin[e], &cur, p, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
            }
        }
    }
    for (uint64_t j = 0; j < ns; j++) {
        int r = 0;
        for (int t = 0; t < k - 1 && !r; t++) {
            const uint64_t b = (uint64_t)sidx[j * 64 + t];
            uint64_t e = (b * 0x9E3779B97F4A7C15ull) >> (64 - lg);
            while (tbit[e] != b) e = (e + 1) & (cap - 1);
            r = tmin[e] == sample[j] * (uint64_t)k + (uint64_t)t;
        }
        out[j] = (uint8_t)r;
    }
    free(tbit);
    free(tmin);
    free(scr);
    free(sidx);
    (void)nthreads;
}

/* contains(), RedissonBloomFilter.java:133-168: AND over getbit_0..getbit_{k-2}. */
void orc_bloom_contains_batch(const uint8_t *bits, int64_t size, int k, const uint8_t *data,
                              const uint64_t *offsets, uint32_t fixed_len, uint64_t n, uint8_t *out) {
    int64_t idx[64];
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p = offsets ? data + offsets[i] : data + i * (uint64_t)fixed_len;
        size_t len = offsets ? (size_t)(offsets[i + 1] - offsets[i]) : fixed_len;
        orc_bloom_indexes(p, len, k, size, idx);
        int r = 1;
        for (int t = 0; t < k - 1; t++)
            if (!orc_getbit(bits, (uint64_t)idx[t])) { r = 0; break; }
        out[i] = (uint8_t)r;
    }
}
