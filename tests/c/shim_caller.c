/*
 * shim_caller.c -- drives librsketch.so through the Java binding's shim
 * (jni/rsketch_shim.c) exactly as jni/rsketch_jni.c does: "direct buffers"
 * (plain host memory + capacity), names, jlong space handle, boolean[] reply
 * regions, status -> exception class, completion callbacks.  Replays the
 * reference's JUnit cases (src/test/java/org/redisson/RedissonHyperLogLogTest.java:
 * 10-38, RedissonBloomFilterTest.java:10-66) -- the IllegalStateException of
 * every getter and of add/contains on a filter nobody initialised, tryInit's
 * idempotence ACROSS instances (two lookups of one name = one filter), count
 * of a missing HLL creating nothing, the "config has been changed" guard --
 * then the RBatch of add()s, async calls from two threads on two handles,
 * completion callbacks that call back into the shim (a further async add and
 * a synchronous count from inside a callback, a delete whose last reference
 * drops in a callback, a callback's call while another thread waits in
 * rsk_shim_sync -- none may deadlock: a watchdog fails the run), RBitSet on a
 * plain name and on a Bloom filter's name (getBitSet(filterName) reads the
 * filter's bits: GET equals rsk_bloom_export_bits up to Redis's STRLEN), and a
 * 200k-element batch checked against the CPU oracle.  Needs a GPU; run by
 * tests/test_jni_shim.py (-m gpu).
 * Exit 0 = all checks passed; prints one line per failed check otherwise.
 */
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

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

static int64_t S; /* the space: one GPU context + its keyspace */

/* hll.add(e): one PFADD of one JsonJacksonCodec-encoded element */
static int hll_add1(const char *name, const char *json, uint8_t *changed) {
  batch b = {.n = 0};
  put(&b, json);
  return rsk_shim_hll_add(S, name, kbuf(&b), obuf(&b), 1, changed);
}

/* A GpuBloomFilter instance: its cached (size, k), as RedissonBloomFilter
 * keeps size / hashIterations (:54-55) and re-reads them when 0 or stale. */
typedef struct {
  const char *name;
  int64_t size;
  int32_t k;
} bloom_obj;

static int read_config(bloom_obj *o) {
  rsk_shim_bloom_config c;
  int rc = rsk_shim_bloom_get_config(S, o->name, &c);
  if (rc == RSK_OK) {
    o->size = c.size;
    o->k = c.hash_iterations;
  }
  return rc;
}

/* add(obj) / contains(obj) with the reference's retry loop (:83-113). */
static int bloom_call(bloom_obj *o, const char *json, uint8_t *r, int add, int *retries) {
  batch b = {.n = 0};
  put(&b, json);
  for (;;) {
    if (o->size == 0) {
      int rc = read_config(o);
      if (rc) return rc;
    }
    int rc = add ? rsk_shim_bloom_add(S, o->name, o->size, o->k, kbuf(&b), obuf(&b), 1, r, 1)
                 : rsk_shim_bloom_contains(S, o->name, o->size, o->k, kbuf(&b), obuf(&b), 1, r, 1);
    if (rc != RSK_SHIM_CONFIG_CHANGED) return rc;
    if (retries) ++*retries;
    o->size = 0; /* re-read {name}__config and try again */
  }
}

/* ------------------------------------------------------------- async */
typedef struct {
  pthread_mutex_t mu;
  pthread_cond_t cv;
  int fired[64];
  uint64_t value[64];
  int status[64];
} waiter;
static waiter W = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, {0}, {0}, {0}};

static void done(void *user, int status, uint64_t value) {
  const int slot = (int)(intptr_t)user;
  pthread_mutex_lock(&W.mu);
  W.fired[slot] += 1;
  W.value[slot] = value;
  W.status[slot] = status;
  pthread_cond_broadcast(&W.cv);
  pthread_mutex_unlock(&W.mu);
}

static void wait_slots(int lo, int hi) {
  pthread_mutex_lock(&W.mu);
  for (;;) {
    int all = 1;
    for (int i = lo; i < hi; ++i) all &= W.fired[i] > 0;
    if (all) break;
    pthread_cond_wait(&W.cv, &W.mu);
  }
  pthread_mutex_unlock(&W.mu);
}

typedef struct {
  const char *name;
  unsigned char *keys;
  int64_t *offs;
  int64_t n;
  int slot0;
  int rc;
} async_job;

static void *issue(void *p) {
  async_job *j = p;
  j->rc = RSK_OK;
  for (int r = 0; r < 3 && j->rc == RSK_OK; ++r) /* first creates the key (1), repeats change nothing (0) */
    j->rc = rsk_shim_hll_add_async(S, j->name, (rsk_shim_buf){j->keys, 16 * j->n}, (rsk_shim_buf){j->offs, j->n + 1},
                                   j->n, done, (void *)(intptr_t)(j->slot0 + r));
  return NULL;
}

/* ------------------------------------------------- re-entrant callbacks */
static batch RE; /* the keys the callbacks add */
static volatile int re_rc_async = -1, re_rc_count = -1;
static volatile int64_t re_count = -1;

/* Slot 40: from inside the completion, issue a further async add (slot 41)
 * and a synchronous count on the same space. */
static void reenter(void *user, int status, uint64_t value) {
  (void)user;
  (void)status;
  (void)value;
  re_rc_async = rsk_shim_hll_add_async(S, "reent", kbuf(&RE), obuf(&RE), 2, done, (void *)(intptr_t)41);
  int64_t c = -1;
  re_rc_count = rsk_shim_hll_count(S, "reent", &c);
  re_count = c;
  done((void *)(intptr_t)40, status, value);
}

/* Slot 42: waits until the main thread is (about to be) inside
 * rsk_shim_sync, then makes a synchronous library call -- the round-3 code
 * held the context lock while waiting for this callback. */
static volatile int sync_started;
static void late_caller(void *user, int status, uint64_t value) {
  (void)user;
  while (!sync_started) {
    const struct timespec ts = {0, 1000000L};
    nanosleep(&ts, NULL);
  }
  const struct timespec ts = {0, 50000000L}; /* 50 ms: the main thread is inside the wait by now */
  nanosleep(&ts, NULL);
  int64_t c = -1;
  const int rc = rsk_shim_hll_count(S, "reent", &c);
  done((void *)(intptr_t)42, rc == RSK_OK ? status : rc, (uint64_t)c);
  (void)value;
}

/* Slot 43: deletes the name its own call went to -- the map's reference is
 * the last one, so the sketch is destroyed from inside the callback. */
static void deleter(void *user, int status, uint64_t value) {
  (void)user;
  int32_t d = -1;
  const int rc = rsk_shim_delete(S, "doomed", &d);
  done((void *)(intptr_t)43, rc == RSK_OK && d == 1 ? status : 99, value);
}

static void on_alarm(int sig) {
  (void)sig;
  static const char msg[] = "FAIL watchdog: a call deadlocked\n";
  (void)!write(2, msg, sizeof msg - 1);
  _exit(3);
}

static int contains_bytes(const uint8_t *a, size_t na, const uint8_t *b, size_t nb) {
  return na == nb && (na == 0 || memcmp(a, b, na) == 0);
}

int main(void) {
  signal(SIGALRM, on_alarm);
  alarm(100); /* every check below finishes in seconds; a deadlock does not */
  if (rsk_shim_init(0, 0, &S)) {
    fprintf(stderr, "init: %s (%s)\n", rsk_shim_last_error(), rsk_shim_exception_class(RSK_ERR_NO_DEVICE));
    return 2;
  }
  uint8_t ch = 0;
  int64_t cnt = -1;
  int32_t type = -1;
  int64_t hnd = 0, hnd2 = 0;

  /* RedissonHyperLogLogTest.testAdd: Integers 1, 2, 3 (Jackson "1","2","3") -> count 3 */
  CHECK(hll_add1("log", "1", &ch) == RSK_OK && ch == 1);
  CHECK(hll_add1("log", "2", &ch) == RSK_OK && ch == 1);
  CHECK(hll_add1("log", "3", &ch) == RSK_OK && ch == 1);
  CHECK(rsk_shim_hll_count(S, "log", &cnt) == RSK_OK && cnt == 3);

  /* testMerge: replies true x4, true x3, false for the repeated "c"; merge -> 6 */
  const char *a1[] = {"\"foo\"", "\"bar\"", "\"zap\"", "\"a\""};
  for (int i = 0; i < 4; ++i) CHECK(hll_add1("hll1", a1[i], &ch) == RSK_OK && ch == 1);
  const char *a2[] = {"\"a\"", "\"b\"", "\"c\"", "\"foo\""};
  for (int i = 0; i < 4; ++i) CHECK(hll_add1("hll2", a2[i], &ch) == RSK_OK && ch == 1);
  CHECK(hll_add1("hll2", "\"c\"", &ch) == RSK_OK && ch == 0);
  const char *srcs[] = {"hll1", "hll2"};
  CHECK(rsk_shim_hll_merge_with(S, "hll3", srcs, 2) == RSK_OK);
  CHECK(rsk_shim_hll_count(S, "hll3", &cnt) == RSK_OK && cnt == 6);
  CHECK(rsk_shim_hll_count_with(S, srcs, 2, &cnt) == RSK_OK && cnt == 6);

  /* PFCOUNT of a missing key: 0, and the key stays missing (no creation) */
  CHECK(rsk_shim_hll_count(S, "nobody", &cnt) == RSK_OK && cnt == 0);
  CHECK(rsk_shim_lookup(S, "nobody", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE && hnd == 0);
  const char *with_missing[] = {"hll1", "nobody", "hll2"};
  CHECK(rsk_shim_hll_count_with(S, with_missing, 3, &cnt) == RSK_OK && cnt == 6);
  CHECK(rsk_shim_lookup(S, "nobody", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE);
  /* two lookups of one name are one key (one handle) */
  CHECK(rsk_shim_lookup(S, "hll1", &type, &hnd) == RSK_OK && type == RSK_SHIM_HLL && hnd != 0);
  CHECK(rsk_shim_lookup(S, "hll1", &type, &hnd2) == RSK_OK && hnd2 == hnd);
  const int64_t h_hll1 = hnd;
  /* PFMERGE into a new key from a missing source only: the key exists, empty */
  const char *only_missing[] = {"nobody"};
  CHECK(rsk_shim_hll_merge_with(S, "merged-empty", only_missing, 1) == RSK_OK);
  CHECK(rsk_shim_lookup(S, "merged-empty", &type, &hnd) == RSK_OK && type == RSK_SHIM_HLL);
  CHECK(rsk_shim_hll_count(S, "merged-empty", &cnt) == RSK_OK && cnt == 0);
  int32_t deleted = 0, renamed = -1;
  /* RENAME / RENAMENX move the key; the sketch follows its name */
  CHECK(rsk_shim_rename(S, "hll1", "hll1b", 0, &renamed) == RSK_OK && renamed == 1);
  CHECK(rsk_shim_lookup(S, "hll1", &type, &hnd2) == RSK_OK && type == RSK_SHIM_NONE);
  CHECK(rsk_shim_lookup(S, "hll1b", &type, &hnd2) == RSK_OK && type == RSK_SHIM_HLL && hnd2 == h_hll1);
  CHECK(rsk_shim_hll_count(S, "hll1b", &cnt) == RSK_OK && cnt == 4);
  CHECK(rsk_shim_rename(S, "hll1b", "hll2", 1, &renamed) == RSK_OK && renamed == 0); /* NX onto a key: no */
  CHECK(rsk_shim_rename(S, "nobody", "x", 0, &renamed) == RSK_ERR_INVALID_ARG);
  CHECK(rsk_shim_rename(S, "hll1b", "hll1", 0, &renamed) == RSK_OK && renamed == 1);
  CHECK(rsk_shim_delete(S, "merged-empty", &deleted) == RSK_OK && deleted == 1);
  CHECK(rsk_shim_delete(S, "merged-empty", &deleted) == RSK_OK && deleted == 0);

  /* add() as RBatch: one PFADD per element, replies in order, across names */
  {
    batch b = {.n = 0};
    put(&b, "\"x\"");
    put(&b, "\"y\"");
    put(&b, "\"x\"");
    put(&b, "\"x\"");
    put(&b, "\"z\"");
    uint8_t rep[5] = {9, 9, 9, 9, 9};
    CHECK(rsk_shim_hll_add_each(S, "each", kbuf(&b), obuf(&b), 3, rep, 3) == RSK_OK);
    CHECK(rep[0] == 1 && rep[1] == 1 && rep[2] == 0);
    CHECK(rsk_shim_hll_add_each(S, "each", kbuf(&b), obuf(&b), 3, rep, 2) == RSK_ERR_INVALID_ARG);
    /* batch: x->A, y->B, x->A (repeat: 0), x->B (new in B: 1), z->A */
    const char *names[] = {"batchA", "batchB"};
    const int32_t name_of[5] = {0, 1, 0, 1, 0};
    memset(rep, 9, sizeof rep);
    CHECK(rsk_shim_batch_hll_add(S, names, 2, name_of, kbuf(&b), obuf(&b), 5, rep, 5) == RSK_OK);
    CHECK(rep[0] == 1 && rep[1] == 1 && rep[2] == 0 && rep[3] == 1 && rep[4] == 1);
    CHECK(rsk_shim_hll_count(S, "batchA", &cnt) == RSK_OK && cnt == 2);
    CHECK(rsk_shim_hll_count(S, "batchB", &cnt) == RSK_OK && cnt == 2);
    const int32_t bad_of[5] = {0, 1, 2, 0, 0};
    CHECK(rsk_shim_batch_hll_add(S, names, 2, bad_of, kbuf(&b), obuf(&b), 5, rep, 5) == RSK_ERR_INVALID_ARG);
  }

  /* bad "direct buffers" stop in the shim: IllegalArgumentException, no device access */
  {
    batch b = {.n = 0};
    put(&b, "\"a\"");
    put(&b, "\"b\"");
    rsk_shim_buf small = {b.bytes, 4}; /* offsets reach 6 */
    CHECK(rsk_shim_hll_add(S, "log", small, obuf(&b), 2, &ch) == RSK_ERR_INVALID_ARG);
    CHECK(strcmp(rsk_shim_exception_class(RSK_ERR_INVALID_ARG), "java/lang/IllegalArgumentException") == 0);
    CHECK(strstr(rsk_shim_last_error(), "past the keys buffer") != NULL);
    rsk_shim_buf few = {b.offs, 2}; /* n+1 = 3 offsets needed */
    CHECK(rsk_shim_hll_add(S, "log", kbuf(&b), few, 2, &ch) == RSK_ERR_INVALID_ARG);
    rsk_shim_buf heap = {NULL, 0}; /* a heap ByteBuffer: GetDirectBufferAddress == NULL */
    CHECK(rsk_shim_hll_add(S, "log", kbuf(&b), heap, 2, &ch) == RSK_ERR_INVALID_ARG);
    int64_t dec[3] = {0, 3, 2};
    rsk_shim_buf decb = {dec, 3};
    CHECK(rsk_shim_hll_add(S, "log", kbuf(&b), decb, 2, &ch) == RSK_ERR_INVALID_ARG);
    CHECK(rsk_shim_hll_count(S, "log", &cnt) == RSK_OK && cnt == 3); /* untouched */
  }

  /* RedissonBloomFilterTest.testConfig: tryInit(100, 0.03) -> the four getters */
  int32_t created = -1;
  rsk_shim_bloom_config cfg;
  CHECK(rsk_shim_bloom_try_init(S, "filter", 100, 0.03, &created, &cfg) == RSK_OK && created == 1);
  CHECK(rsk_shim_bloom_get_config(S, "filter", &cfg) == RSK_OK);
  CHECK(cfg.expected_insertions == 100 && cfg.false_probability == 0.03 && cfg.hash_iterations == 5 &&
        cfg.size == 729);
  CHECK(rsk_shim_delete(S, "filter", &deleted) == RSK_OK && deleted == 1);

  /* testInit: idempotent (false the second time, also from a second instance
   * whose arguments differ), true again after delete() */
  CHECK(rsk_shim_bloom_try_init(S, "filter", 55000000LL, 0.03, &created, NULL) == RSK_OK && created == 1);
  CHECK(rsk_shim_bloom_try_init(S, "filter", 55000001LL, 0.03, &created, &cfg) == RSK_OK && created == 0);
  CHECK(cfg.expected_insertions == 55000000LL); /* the stored config, not the second caller's */
  {
    bloom_obj second = {"filter", 0, 0}; /* another getBloomFilter("filter") */
    CHECK(read_config(&second) == RSK_OK && second.size == cfg.size && second.k == cfg.hash_iterations);
  }
  CHECK(rsk_shim_delete(S, "filter", &deleted) == RSK_OK && deleted == 1);
  CHECK(rsk_shim_bloom_try_init(S, "filter", 55000001LL, 0.03, &created, NULL) == RSK_OK && created == 1);
  CHECK(rsk_shim_delete(S, "filter", &deleted) == RSK_OK && deleted == 1);

  /* testNotInitializedOnExpectedInsertions / OnContains / OnAdd: IllegalStateException */
  {
    CHECK(rsk_shim_bloom_get_config(S, "filter", &cfg) == RSK_ERR_NOT_INITIALIZED);
    CHECK(strcmp(rsk_shim_exception_class(RSK_ERR_NOT_INITIALIZED), "java/lang/IllegalStateException") == 0);
    CHECK(strcmp(rsk_shim_last_error(), "Bloom filter is not initialized!") == 0);
    bloom_obj f = {"filter", 0, 0};
    uint8_t r = 9;
    CHECK(bloom_call(&f, "\"32\"", &r, 0, NULL) == RSK_ERR_NOT_INITIALIZED);
    CHECK(bloom_call(&f, "\"123\"", &r, 1, NULL) == RSK_ERR_NOT_INITIALIZED);
    int32_t bc = -1;
    CHECK(rsk_shim_bloom_count(S, "filter", &bc) == RSK_ERR_NOT_INITIALIZED);
    CHECK(rsk_shim_lookup(S, "filter", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE); /* nothing created */
  }

  /* oversize tryInit refused in compat mode before the keyspace is looked at */
  CHECK(rsk_shim_bloom_try_init(S, "big", 1000000000LL, 0.01, &created, NULL) == RSK_ERR_INVALID_ARG);
  CHECK(rsk_shim_lookup(S, "big", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE);

  /* RedissonBloomFilterTest.test: tryInit(550000000, 0.03) and the replies */
  {
    bloom_obj f = {"filter", 0, 0};
    CHECK(rsk_shim_bloom_try_init(S, "filter", 550000000LL, 0.03, &created, &cfg) == RSK_OK && created == 1);
    CHECK(cfg.size == 4014142460LL && cfg.hash_iterations == 5);
    uint8_t r = 9;
    int32_t bc = -1;
    const char *s2 = "\"hflgs;jl;ao1-32471320o31803-24\"";
    CHECK(bloom_call(&f, "\"123\"", &r, 0, NULL) == RSK_OK && r == 0);
    CHECK(bloom_call(&f, "\"123\"", &r, 1, NULL) == RSK_OK && r == 1);
    CHECK(bloom_call(&f, "\"123\"", &r, 0, NULL) == RSK_OK && r == 1);
    CHECK(bloom_call(&f, "\"123\"", &r, 1, NULL) == RSK_OK && r == 0);
    CHECK(rsk_shim_bloom_count(S, "filter", &bc) == RSK_OK && bc == 1);
    CHECK(bloom_call(&f, s2, &r, 0, NULL) == RSK_OK && r == 0);
    CHECK(bloom_call(&f, s2, &r, 1, NULL) == RSK_OK && r == 1);
    CHECK(bloom_call(&f, s2, &r, 0, NULL) == RSK_OK && r == 1);
    CHECK(rsk_shim_bloom_count(S, "filter", &bc) == RSK_OK && bc == 2);
    /* a name holding a Bloom filter is not an HLL */
    CHECK(hll_add1("filter", "1", &ch) == RSK_ERR_WRONGTYPE);
    CHECK(rsk_shim_hll_count(S, "filter", &cnt) == RSK_ERR_WRONGTYPE);

    /* config changed under an instance: another client deletes and re-inits
     * with other parameters; the stale (size, k) is refused
     * (RSK_SHIM_CONFIG_CHANGED -> RedisException "...config has been changed"),
     * the instance re-reads {name}__config and its retry succeeds */
    CHECK(rsk_shim_delete(S, "filter", &deleted) == RSK_OK && deleted == 1);
    CHECK(rsk_shim_bloom_try_init(S, "filter", 1000, 0.01, &created, &cfg) == RSK_OK && created == 1);
    batch b = {.n = 0};
    put(&b, "\"123\"");
    CHECK(rsk_shim_bloom_add(S, "filter", 4014142460LL, 5, kbuf(&b), obuf(&b), 1, &r, 1) == RSK_SHIM_CONFIG_CHANGED);
    CHECK(strcmp(rsk_shim_exception_class(RSK_SHIM_CONFIG_CHANGED), "org/redisson/client/RedisException") == 0);
    CHECK(strstr(rsk_shim_last_error(), "Bloom filter config has been changed") != NULL);
    int retries = 0;
    CHECK(bloom_call(&f, "\"123\"", &r, 1, &retries) == RSK_OK && r == 1 && retries == 1);
    CHECK(f.size == cfg.size && f.k == cfg.hash_iterations && f.k == 7);
    CHECK(rsk_shim_delete(S, "filter", &deleted) == RSK_OK && deleted == 1);
  }

  /* async: two threads issue adds on two names at once; every callback fires
   * once with the right reply, and the sketches equal the oracle's */
  {
    const int64_t n = 100000;
    async_job jobs[2];
    unsigned char *keys[2];
    int64_t *offs = malloc((size_t)(n + 1) * 8);
    for (int64_t i = 0; i <= n; ++i) offs[i] = 16 * i;
    for (int t = 0; t < 2; ++t) {
      keys[t] = malloc((size_t)n * 16);
      orc_gen_keys16(0x5EED0100 + t, 0, (uint64_t)n, keys[t]);
      jobs[t] = (async_job){t ? "asyncB" : "asyncA", keys[t], offs, n, 10 * t, -1};
    }
    pthread_t th[2];
    for (int t = 0; t < 2; ++t) pthread_create(&th[t], NULL, issue, &jobs[t]);
    for (int t = 0; t < 2; ++t) pthread_join(th[t], NULL);
    CHECK(jobs[0].rc == RSK_OK && jobs[1].rc == RSK_OK);
    wait_slots(0, 3);
    wait_slots(10, 13);
    for (int t = 0; t < 2; ++t)
      for (int r = 0; r < 3; ++r) {
        const int sl = 10 * t + r;
        CHECK(W.fired[sl] == 1 && W.status[sl] == RSK_OK && W.value[sl] == (r == 0 ? 1u : 0u));
      }
    /* countAsync on both, and on a missing name (fires at once with 0) */
    CHECK(rsk_shim_hll_count_async(S, "asyncA", done, (void *)(intptr_t)20) == RSK_OK);
    CHECK(rsk_shim_hll_count_async(S, "asyncB", done, (void *)(intptr_t)21) == RSK_OK);
    CHECK(rsk_shim_hll_count_async(S, "nobody", done, (void *)(intptr_t)22) == RSK_OK);
    const char *ab[] = {"asyncA", "asyncB"};
    CHECK(rsk_shim_hll_merge_with_async(S, "asyncAB", ab, 2, done, (void *)(intptr_t)23) == RSK_OK);
    CHECK(rsk_shim_hll_count_with_async(S, ab, 2, done, (void *)(intptr_t)24) == RSK_OK);
    wait_slots(20, 25);
    for (int t = 0; t < 2; ++t) {
      uint8_t *regs = calloc(16384, 1);
      orc_hll_add_raw(regs, keys[t], NULL, 16, (uint64_t)n);
      CHECK(W.value[20 + t] == orc_hll_count_dense_regs(regs));
      free(regs);
    }
    CHECK(W.fired[22] == 1 && W.value[22] == 0);
    CHECK(rsk_shim_lookup(S, "nobody", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE);
    int64_t ab_count = -1;
    CHECK(rsk_shim_hll_count(S, "asyncAB", &ab_count) == RSK_OK && W.value[24] == (uint64_t)ab_count);
    /* delete while nothing is in flight, then async Bloom add + contains */
    CHECK(rsk_shim_delete(S, "asyncAB", &deleted) == RSK_OK && deleted == 1);
    CHECK(rsk_shim_bloom_try_init(S, "abloom", n, 0.01, &created, &cfg) == RSK_OK && created == 1);
    uint8_t *got = malloc((size_t)n), *want = malloc((size_t)n), *con = malloc((size_t)n);
    unsigned char *bits = calloc((size_t)((cfg.size + 7) / 8), 1);
    rsk_shim_buf kb = {keys[0], 16 * n}, ob = {offs, n + 1};
    CHECK(rsk_shim_bloom_add_async(S, "abloom", cfg.size, cfg.hash_iterations, kb, ob, n, got, n, done,
                                   (void *)(intptr_t)30) == RSK_OK);
    CHECK(rsk_shim_bloom_contains_async(S, "abloom", cfg.size, cfg.hash_iterations, kb, ob, n, con, n, done,
                                        (void *)(intptr_t)31) == RSK_OK);
    /* the filter is deleted while both calls may still run: they finish first */
    CHECK(rsk_shim_delete(S, "abloom", &deleted) == RSK_OK && deleted == 1);
    wait_slots(30, 32);
    CHECK(W.value[30] == (uint64_t)n && W.value[31] == (uint64_t)n);
    orc_bloom_add_batch(bits, cfg.size, cfg.hash_iterations, keys[0], NULL, 16, (uint64_t)n, want);
    CHECK(memcmp(got, want, (size_t)n) == 0);
    int all = 1;
    for (int64_t i = 0; i < n; ++i) all &= con[i] == 1;
    CHECK(all);
    free(got), free(want), free(con), free(bits), free(offs);
    free(keys[0]), free(keys[1]);
  }

  /* Completion callbacks that call back into the shim. */
  {
    put(&RE, "\"r1\"");
    put(&RE, "\"r2\"");
    CHECK(rsk_shim_hll_add_async(S, "reent", kbuf(&RE), obuf(&RE), 1, reenter, NULL) == RSK_OK);
    wait_slots(40, 42);
    CHECK(re_rc_async == RSK_OK && re_rc_count == RSK_OK && re_count >= 1);
    CHECK(W.value[40] == 1 && W.value[41] == 1); /* "r1" created the key; "r2" grew it */
    CHECK(rsk_shim_hll_count(S, "reent", &cnt) == RSK_OK && cnt == 2);

    /* a callback's synchronous call while the main thread waits in rsk_shim_sync */
    CHECK(rsk_shim_hll_add_async(S, "reent", kbuf(&RE), obuf(&RE), 2, late_caller, NULL) == RSK_OK);
    sync_started = 1;
    CHECK(rsk_shim_sync(S) == RSK_OK);
    CHECK(W.fired[42] == 1 && W.status[42] == RSK_OK && W.value[42] == 2); /* sync waited for the callback */

    /* the last reference drops inside the callback (the callback deletes) */
    CHECK(rsk_shim_hll_add_async(S, "doomed", kbuf(&RE), obuf(&RE), 2, deleter, NULL) == RSK_OK);
    wait_slots(43, 44);
    CHECK(W.status[43] == RSK_OK);
    CHECK(rsk_shim_lookup(S, "doomed", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE);
    /* ... and the last reference drops in the shim's own completion (delete while in flight) */
    CHECK(rsk_shim_hll_add_async(S, "doomed2", kbuf(&RE), obuf(&RE), 2, done, (void *)(intptr_t)44) == RSK_OK);
    CHECK(rsk_shim_delete(S, "doomed2", &deleted) == RSK_OK && deleted == 1);
    wait_slots(44, 45);
    CHECK(rsk_shim_sync(S) == RSK_OK);
    CHECK(rsk_shim_lookup(S, "doomed2", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE);
  }

  /* RBitSet on plain names (RedissonBitSetTest.java:12-137 semantics) */
  {
    int64_t v = -1;
    uint8_t *bytes = NULL;
    int64_t len = 0;
    CHECK(rsk_shim_bitset_get_bytes(S, "bs", &bytes, &len) == RSK_OK && len == -1 && !bytes); /* nil */
    CHECK(rsk_shim_bitset_cardinality(S, "bs", &v) == RSK_OK && v == 0);
    const int64_t idx[3] = {3, 5, 17};
    CHECK(rsk_shim_bitset_setbits(S, "bs", idx, 3, 1) == RSK_OK);
    CHECK(rsk_shim_bitset_strlen(S, "bs", &v) == RSK_OK && v == 3); /* (17 >> 3) + 1 */
    CHECK(rsk_shim_bitset_cardinality(S, "bs", &v) == RSK_OK && v == 3);
    CHECK(rsk_shim_bitset_length(S, "bs", &v) == RSK_OK && v == 18);
    CHECK(rsk_shim_bitset_get_bytes(S, "bs", &bytes, &len) == RSK_OK && len == 3);
    if (len == 3) CHECK(bytes[0] == 0x14 && bytes[1] == 0 && bytes[2] == 0x40); /* MSB-first */
    rsk_shim_free(bytes);
    uint8_t g[4];
    const int64_t q[4] = {3, 4, 17, 100000};
    CHECK(rsk_shim_bitset_getbits(S, "bs", q, 4, g, 4) == RSK_OK && g[0] == 1 && g[1] == 0 && g[2] == 1 && g[3] == 0);
    const int64_t bad[1] = {-1};
    CHECK(rsk_shim_bitset_setbits(S, "bs", bad, 1, 1) == RSK_SHIM_REDIS_ERROR);
    CHECK(strcmp(rsk_shim_exception_class(RSK_SHIM_REDIS_ERROR), "org/redisson/client/RedisException") == 0);
    /* BITOP AND bs bs other (RedissonBitSetTest.testAnd): other missing -> empty -> bs goes away */
    const char *other[1] = {"bs-other"};
    CHECK(rsk_shim_bitset_set_range(S, "bs-other", 0, 8, 1) == RSK_OK); /* byte 0 = 0xFF */
    CHECK(rsk_shim_bitset_op(S, "bs", RSK_BITOP_AND, other, 1) == RSK_OK);
    CHECK(rsk_shim_bitset_get_bytes(S, "bs", &bytes, &len) == RSK_OK && len == 3);
    if (len == 3) CHECK(bytes[0] == 0x14 && bytes[1] == 0 && bytes[2] == 0);
    rsk_shim_free(bytes);
    const char *nobody[1] = {"bs-nobody"};
    CHECK(rsk_shim_bitset_op(S, "bs-new", RSK_BITOP_OR, nobody, 1) == RSK_OK); /* all empty: no key */
    CHECK(rsk_shim_lookup(S, "bs-new", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE);
    CHECK(rsk_shim_bitset_op(S, "bs", RSK_BITOP_NOT, other, 1) == RSK_SHIM_REDIS_ERROR);
    int32_t dd = 0;
    CHECK(rsk_shim_bitset_clear(S, "bs", &dd) == RSK_OK && dd == 1);
    CHECK(rsk_shim_lookup(S, "bs", &type, &hnd) == RSK_OK && type == RSK_SHIM_NONE);
    CHECK(rsk_shim_bitset_cardinality(S, "log", &v) == RSK_ERR_WRONGTYPE); /* an HLL name */
    CHECK(rsk_shim_delete(S, "bs-other", &deleted) == RSK_OK && deleted == 1);
  }

  /* getBitSet(bloomName): the filter's bits, as Redis's GET of the filter key */
  {
    const int64_t n = 20000;
    unsigned char *keys = malloc((size_t)n * 16);
    int64_t *offs = malloc((size_t)(n + 1) * 8);
    orc_gen_keys16(0x5EED0200, 0, (uint64_t)n, keys);
    for (int64_t i = 0; i <= n; ++i) offs[i] = 16 * i;
    rsk_shim_buf kb = {keys, 16 * n}, ob = {offs, n + 1};
    CHECK(rsk_shim_bloom_try_init(S, "bf", n, 0.01, &created, &cfg) == RSK_OK && created == 1);
    uint8_t *bytes = NULL;
    int64_t len = 0, v = -1;
    CHECK(rsk_shim_bitset_get_bytes(S, "bf", &bytes, &len) == RSK_OK && len == -1); /* nothing added: no string */
    CHECK(rsk_shim_bloom_add(S, "bf", cfg.size, cfg.hash_iterations, kb, ob, n, NULL, 0) == RSK_OK);
    CHECK(rsk_shim_lookup(S, "bf", &type, &hnd) == RSK_OK && type == RSK_SHIM_BLOOM);
    const size_t nb = (size_t)((cfg.size + 7) / 8);
    uint8_t *exp = malloc(nb);
    size_t elen = 0;
    CHECK(rsk_bloom_export_bits((rsk_bloom *)(intptr_t)hnd, exp, nb, &elen) == RSK_OK && elen == nb);
    size_t redis_len = elen; /* STRLEN: the last byte a SETBIT touched (adds only set bits) */
    while (redis_len > 0 && exp[redis_len - 1] == 0) --redis_len;
    CHECK(rsk_shim_bitset_get_bytes(S, "bf", &bytes, &len) == RSK_OK);
    CHECK(contains_bytes(bytes, (size_t)len, exp, redis_len));
    rsk_shim_free(bytes);
    CHECK(rsk_shim_bitset_strlen(S, "bf", &v) == RSK_OK && v == (int64_t)redis_len);
    uint64_t pc = 0;
    for (size_t i = 0; i < nb; ++i) pc += (uint64_t)__builtin_popcount(exp[i]);
    CHECK(rsk_shim_bitset_cardinality(S, "bf", &v) == RSK_OK && (uint64_t)v == pc);
    /* the oracle's bit string for the same adds */
    uint8_t *obits = calloc(nb, 1);
    orc_bloom_add_batch(obits, cfg.size, cfg.hash_iterations, keys, NULL, 16, (uint64_t)n, NULL);
    CHECK(memcmp(obits, exp, nb) == 0);
    /* GETBIT of the first set bit and of a clear one */
    int64_t first = -1, clear = -1;
    for (int64_t i = 0; i < (int64_t)nb * 8 && (first < 0 || clear < 0); ++i) {
      const int set = (exp[i >> 3] >> (7 - (i & 7))) & 1;
      if (set && first < 0) first = i;
      if (!set && clear < 0) clear = i;
    }
    const int64_t q[2] = {first, clear};
    uint8_t g[2] = {9, 9};
    CHECK(rsk_shim_bitset_getbits(S, "bf", q, 2, g, 2) == RSK_OK && g[0] == 1 && g[1] == 0);
    /* a write through the RBitSet is a write to the filter: clear() = DEL of the
     * string; the filter stays initialised (its {name}__config) with no bits */
    int32_t dd = 0, bc = -1;
    CHECK(rsk_shim_bitset_clear(S, "bf", &dd) == RSK_OK && dd == 1);
    CHECK(rsk_shim_bloom_count(S, "bf", &bc) == RSK_OK && bc == 0);
    CHECK(rsk_shim_bloom_get_config(S, "bf", &cfg) == RSK_OK);
    CHECK(rsk_shim_bitset_strlen(S, "bf", &v) == RSK_OK && v == 0);
    CHECK(rsk_shim_delete(S, "bf", &deleted) == RSK_OK && deleted == 1);
    free(keys), free(offs), free(exp), free(obits);
  }

  /* A 200k-element addAll through one "direct buffer" pair against the oracle. */
  {
    const int64_t n = 200000;
    unsigned char *keys = malloc((size_t)n * 16);
    int64_t *offs = malloc((size_t)(n + 1) * 8);
    orc_gen_keys16(0x5EED0002, 0, (uint64_t)n, keys);
    for (int64_t i = 0; i <= n; ++i) offs[i] = 16 * i;
    rsk_shim_buf kb = {keys, 16 * n}, ob = {offs, n + 1};
    CHECK(rsk_shim_hll_add(S, "big", kb, ob, n, &ch) == RSK_OK && ch == 1);
    uint8_t *regs = calloc(16384, 1);
    orc_hll_add_raw(regs, keys, NULL, 16, (uint64_t)n);
    CHECK(rsk_shim_hll_count(S, "big", &cnt) == RSK_OK && (uint64_t)cnt == orc_hll_count_dense_regs(regs));
    /* and the Bloom side: tryInit(n, 0.01), addAll replies vs the sequential oracle */
    CHECK(rsk_shim_bloom_try_init(S, "bigbloom", n, 0.01, &created, &cfg) == RSK_OK && created == 1);
    uint8_t *got = malloc((size_t)n), *want = malloc((size_t)n);
    unsigned char *bits = calloc((size_t)((cfg.size + 7) / 8), 1);
    CHECK(rsk_shim_bloom_add(S, "bigbloom", cfg.size, cfg.hash_iterations, kb, ob, n, got, n) == RSK_OK);
    orc_bloom_add_batch(bits, cfg.size, cfg.hash_iterations, keys, NULL, 16, (uint64_t)n, want);
    CHECK(memcmp(got, want, (size_t)n) == 0);
    CHECK(rsk_shim_bloom_contains(S, "bigbloom", cfg.size, cfg.hash_iterations, kb, ob, n, got, n) == RSK_OK);
    int all = 1;
    for (int64_t i = 0; i < n; ++i) all &= got[i] == 1;
    CHECK(all);
    free(keys);
    free(offs);
    free(regs);
    free(got);
    free(want);
    free(bits);
  }

  CHECK(rsk_shim_shutdown(S) == RSK_OK);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("shim_caller ok\n");
  return 0;
}
