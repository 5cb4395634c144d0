/*
 * shim_caller.c -- drives librsketch.so through the Java binding's shim
 * (jni/rsketch_shim.c) exactly as jni/rsketch_jni.c does: "direct buffers"
 * (plain host memory + capacity), jlong handles, boolean[] reply regions,
 * status -> exception class.  Replays the reference's JUnit cases
 * (src/test/java/org/redisson/RedissonHyperLogLogTest.java:10-38,
 * RedissonBloomFilterTest.java:10-66) and a 200k-element batch checked against
 * the CPU oracle.  Needs a GPU; run by tests/test_jni_shim.py (-m gpu).
 * Exit 0 = all checks passed; prints one line per failed check otherwise.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../jni/rsketch_shim.h"
#include "../../oracle/rsk_oracle.h"

static int failures;
#define CHECK(cond)                                                  \
  do {                                                               \
    if (!(cond)) {                                                   \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                    \
    }                                                                \
  } while (0)

/* A KeyBuffer (jni/java/org/redisson/gpu/KeyBuffer.java): elements back to
 * back + n+1 native-order offsets. */
typedef struct {
  unsigned char bytes[4096];
  int64_t offs[65];
  int64_t n;
} batch;

static void put(batch *b, const char *s) {
  const size_t l = strlen(s);
  if (b->n == 0) b->offs[0] = 0;
  memcpy(b->bytes + b->offs[b->n], s, l);
  b->offs[b->n + 1] = b->offs[b->n] + (int64_t)l;
  ++b->n;
}

static rsk_shim_buf kbuf(batch *b) { return (rsk_shim_buf){b->bytes, (int64_t)sizeof b->bytes}; }
static rsk_shim_buf obuf(batch *b) { return (rsk_shim_buf){b->offs, 65}; }

/* hll.add(e): one PFADD of one JsonJacksonCodec-encoded element */
static int hll_add1(int64_t h, const char *json, uint8_t *changed) {
  batch b = {.n = 0};
  put(&b, json);
  return rsk_shim_hll_add(h, 0, kbuf(&b), obuf(&b), 1, changed);
}

static int bloom_add1(int64_t bf, const char *json, uint8_t *r) {
  batch b = {.n = 0};
  put(&b, json);
  return rsk_shim_bloom_add(bf, kbuf(&b), obuf(&b), 1, r, 1);
}

static int bloom_contains1(int64_t bf, const char *json, uint8_t *r) {
  batch b = {.n = 0};
  put(&b, json);
  return rsk_shim_bloom_contains(bf, kbuf(&b), obuf(&b), 1, r, 1);
}

int main(void) {
  int64_t ctx = 0;
  if (rsk_shim_init(0, &ctx)) {
    fprintf(stderr, "init: %s (%s)\n", rsk_shim_last_error(), rsk_shim_exception_class(RSK_ERR_NO_DEVICE));
    return 2;
  }
  uint8_t ch = 0;

  /* RedissonHyperLogLogTest.testAdd: Integers 1, 2, 3 (Jackson "1","2","3") -> count 3 */
  int64_t log = 0;
  CHECK(rsk_shim_hll_create(ctx, 1, &log) == RSK_OK);
  CHECK(hll_add1(log, "1", &ch) == RSK_OK && ch == 1);
  CHECK(hll_add1(log, "2", &ch) == RSK_OK && ch == 1);
  CHECK(hll_add1(log, "3", &ch) == RSK_OK && ch == 1);
  int64_t cnt = -1;
  CHECK(rsk_shim_hll_count(log, 0, &cnt) == RSK_OK && cnt == 3);

  /* testMerge: replies true x4, true x3, false for the repeated "c"; merge -> 6 */
  int64_t h1 = 0, h2 = 0, h3 = 0;
  CHECK(rsk_shim_hll_create(ctx, 1, &h1) == RSK_OK);
  CHECK(rsk_shim_hll_create(ctx, 1, &h2) == RSK_OK);
  CHECK(rsk_shim_hll_create(ctx, 1, &h3) == RSK_OK);
  const char *a1[] = {"\"foo\"", "\"bar\"", "\"zap\"", "\"a\""};
  for (int i = 0; i < 4; ++i) CHECK(hll_add1(h1, a1[i], &ch) == RSK_OK && ch == 1);
  const char *a2[] = {"\"a\"", "\"b\"", "\"c\"", "\"foo\""};
  for (int i = 0; i < 4; ++i) CHECK(hll_add1(h2, a2[i], &ch) == RSK_OK && ch == 1);
  CHECK(hll_add1(h2, "\"c\"", &ch) == RSK_OK && ch == 0);
  const int64_t srcs[2] = {h1, h2}, ids[2] = {0, 0};
  CHECK(rsk_shim_hll_merge(h3, 0, srcs, ids, 2) == RSK_OK);
  CHECK(rsk_shim_hll_count(h3, 0, &cnt) == RSK_OK && cnt == 6);
  const int64_t u[2] = {h1, h2};
  CHECK(rsk_shim_hll_count_union(u, ids, 2, &cnt) == RSK_OK && cnt == 6);

  /* add() as RBatch: one PFADD per element, replies in order */
  {
    batch b = {.n = 0};
    put(&b, "\"x\"");
    put(&b, "\"y\"");
    put(&b, "\"x\"");
    uint8_t rep[3] = {9, 9, 9};
    int64_t h4 = 0;
    CHECK(rsk_shim_hll_create(ctx, 1, &h4) == RSK_OK);
    CHECK(rsk_shim_hll_add_each(h4, 0, kbuf(&b), obuf(&b), 3, rep, 3) == RSK_OK);
    CHECK(rep[0] == 1 && rep[1] == 1 && rep[2] == 0);
    CHECK(rsk_shim_hll_add_each(h4, 0, kbuf(&b), obuf(&b), 3, rep, 2) == RSK_ERR_INVALID_ARG);
    CHECK(rsk_shim_hll_destroy(h4) == RSK_OK);
  }

  /* bad "direct buffers" stop in the shim: IllegalArgumentException, no device access */
  {
    batch b = {.n = 0};
    put(&b, "\"a\"");
    put(&b, "\"b\"");
    rsk_shim_buf small = {b.bytes, 4}; /* offsets reach 6 */
    CHECK(rsk_shim_hll_add(log, 0, small, obuf(&b), 2, &ch) == RSK_ERR_INVALID_ARG);
    CHECK(strcmp(rsk_shim_exception_class(RSK_ERR_INVALID_ARG), "java/lang/IllegalArgumentException") == 0);
    CHECK(strstr(rsk_shim_last_error(), "past the keys buffer") != NULL);
    rsk_shim_buf few = {b.offs, 2}; /* n+1 = 3 offsets needed */
    CHECK(rsk_shim_hll_add(log, 0, kbuf(&b), few, 2, &ch) == RSK_ERR_INVALID_ARG);
    rsk_shim_buf heap = {NULL, 0}; /* a heap ByteBuffer: GetDirectBufferAddress == NULL */
    CHECK(rsk_shim_hll_add(log, 0, kbuf(&b), heap, 2, &ch) == RSK_ERR_INVALID_ARG);
    int64_t dec[3] = {0, 3, 2};
    rsk_shim_buf decb = {dec, 3};
    CHECK(rsk_shim_hll_add(log, 0, kbuf(&b), decb, 2, &ch) == RSK_ERR_INVALID_ARG);
    CHECK(rsk_shim_hll_add(log, 1, kbuf(&b), obuf(&b), 2, &ch) == RSK_ERR_INVALID_ARG); /* id out of range */
    CHECK(rsk_shim_hll_count(log, 0, &cnt) == RSK_OK && cnt == 3);                      /* untouched */
  }

  /* RedissonBloomFilterTest.testConfig: tryInit(100, 0.03) -> size 729, k 5;
   * 55000000 @ 0.03 within MAX_SIZE; testInit of a size above MAX_SIZE refused */
  int64_t size = 0;
  int32_t k = 0;
  CHECK(rsk_shim_bloom_params(100, 0.03, 0, &size, &k) == RSK_OK && size == 729 && k == 5);
  CHECK(rsk_shim_bloom_params(550000000LL, 0.03, 0, &size, &k) == RSK_OK && size == 4014142460LL);
  CHECK(rsk_shim_bloom_params(1000000000LL, 0.01, 0, &size, &k) == RSK_ERR_INVALID_ARG);
  CHECK(rsk_shim_bloom_params(1000000000LL, 0.01, 1, &size, &k) == RSK_OK && size == 9585058377LL && k == 7);

  /* testNotInitializedOnAdd: IllegalStateException */
  uint8_t r = 9;
  CHECK(bloom_add1(0, "\"123\"", &r) == RSK_ERR_NOT_INITIALIZED);
  CHECK(strcmp(rsk_shim_exception_class(RSK_ERR_NOT_INITIALIZED), "java/lang/IllegalStateException") == 0);

  /* RedissonBloomFilterTest.test: tryInit(550000000, 0.03) and the replies */
  int64_t bf = 0;
  CHECK(rsk_shim_bloom_params(550000000LL, 0.03, 0, &size, &k) == RSK_OK);
  CHECK(rsk_shim_bloom_create(ctx, size, k, &bf) == RSK_OK);
  int32_t bc = -1;
  const char *s2 = "\"hflgs;jl;ao1-32471320o31803-24\"";
  CHECK(bloom_contains1(bf, "\"123\"", &r) == RSK_OK && r == 0);
  CHECK(bloom_add1(bf, "\"123\"", &r) == RSK_OK && r == 1);
  CHECK(bloom_contains1(bf, "\"123\"", &r) == RSK_OK && r == 1);
  CHECK(bloom_add1(bf, "\"123\"", &r) == RSK_OK && r == 0);
  CHECK(rsk_shim_bloom_count(bf, &bc) == RSK_OK && bc == 1);
  CHECK(bloom_contains1(bf, s2, &r) == RSK_OK && r == 0);
  CHECK(bloom_add1(bf, s2, &r) == RSK_OK && r == 1);
  CHECK(bloom_contains1(bf, s2, &r) == RSK_OK && r == 1);
  CHECK(rsk_shim_bloom_count(bf, &bc) == RSK_OK && bc == 2);
  CHECK(rsk_shim_bloom_destroy(bf) == RSK_OK);

  /* A 200k-element addAll through one "direct buffer" pair against the oracle. */
  {
    const int64_t n = 200000;
    unsigned char *keys = malloc((size_t)n * 16);
    int64_t *offs = malloc((size_t)(n + 1) * 8);
    orc_gen_keys16(0x5EED0002, 0, (uint64_t)n, keys);
    for (int64_t i = 0; i <= n; ++i) offs[i] = 16 * i;
    int64_t big = 0;
    CHECK(rsk_shim_hll_create(ctx, 1, &big) == RSK_OK);
    rsk_shim_buf kb = {keys, 16 * n}, ob = {offs, n + 1};
    CHECK(rsk_shim_hll_add(big, 0, kb, ob, n, &ch) == RSK_OK && ch == 1);
    uint8_t *regs = calloc(16384, 1);
    orc_hll_add_raw(regs, keys, NULL, 16, (uint64_t)n);
    CHECK(rsk_shim_hll_count(big, 0, &cnt) == RSK_OK && (uint64_t)cnt == orc_hll_count_dense_regs(regs));
    /* and the Bloom side: tryInit(n, 0.01), addAll replies vs the sequential oracle */
    CHECK(rsk_shim_bloom_params(n, 0.01, 0, &size, &k) == RSK_OK);
    CHECK(rsk_shim_bloom_create(ctx, size, k, &bf) == RSK_OK);
    uint8_t *got = malloc((size_t)n), *want = malloc((size_t)n);
    unsigned char *bits = calloc((size_t)((size + 7) / 8), 1);
    CHECK(rsk_shim_bloom_add(bf, kb, ob, n, got, n) == RSK_OK);
    orc_bloom_add_batch(bits, size, k, keys, NULL, 16, (uint64_t)n, want);
    CHECK(memcmp(got, want, (size_t)n) == 0);
    CHECK(rsk_shim_bloom_contains(bf, kb, ob, n, got, n) == RSK_OK);
    int all = 1;
    for (int64_t i = 0; i < n; ++i) all &= got[i] == 1;
    CHECK(all);
    CHECK(rsk_shim_bloom_destroy(bf) == RSK_OK);
    CHECK(rsk_shim_hll_destroy(big) == RSK_OK);
    free(keys);
    free(offs);
    free(regs);
    free(got);
    free(want);
    free(bits);
  }

  CHECK(rsk_shim_hll_destroy(log) == RSK_OK);
  CHECK(rsk_shim_hll_destroy(h1) == RSK_OK && rsk_shim_hll_destroy(h2) == RSK_OK && rsk_shim_hll_destroy(h3) == RSK_OK);
  CHECK(rsk_shim_shutdown(ctx) == RSK_OK);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("shim_caller ok\n");
  return 0;
}
