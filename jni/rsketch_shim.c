/*
 * rsketch_shim.c -- argument checks and conversions of the Java binding
 * (see rsketch_shim.h).  Plain C11; links librsketch.so.
 */
#include "rsketch_shim.h"

#include <stdio.h>
#include <string.h>

static _Thread_local char shim_err[256];
static _Thread_local int shim_failed;

static int fail(const char *msg) {
  snprintf(shim_err, sizeof shim_err, "%s", msg);
  shim_failed = 1;
  return RSK_ERR_INVALID_ARG;
}

/* Every entry point clears the shim's own error first; the message the JNI
 * glue reports is the shim's when the shim refused the call, else the
 * library's. */
#define ENTER() (shim_failed = 0)

const char *rsk_shim_last_error(void) { return shim_failed ? shim_err : rsk_last_error(); }

const char *rsk_shim_exception_class(int rc) {
  switch (rc) {
    case RSK_OK:
      return NULL;
    case RSK_ERR_INVALID_ARG:
      return "java/lang/IllegalArgumentException";
    case RSK_ERR_NOT_INITIALIZED:
      return "java/lang/IllegalStateException";
    case RSK_ERR_OUT_OF_MEMORY:
      return "java/lang/OutOfMemoryError";
    default: /* WRONGTYPE, INVALID_HLL, DEVICE, NO_DEVICE */
      return "org/redisson/client/RedisException";
  }
}

int rsk_shim_keys(rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n, rsk_keys *out) {
  if (n < 0) return fail("negative element count");
  memset(out, 0, sizeof *out);
  out->location = RSK_MEM_HOST;
  out->n = (uint64_t)n;
  if (n == 0) return RSK_OK;
  if (!offsets.addr) return fail("offsets must be a direct LongBuffer");
  if (offsets.cap < n + 1) return fail("offsets buffer holds fewer than n+1 longs");
  const int64_t *o = (const int64_t *)offsets.addr;
  if (o[0] < 0) return fail("negative key offset");
  for (int64_t i = 0; i < n; ++i)
    if (o[i + 1] < o[i]) return fail("key offsets decrease");
  if (o[n] > 0 && !keys.addr) return fail("keys must be a direct ByteBuffer");
  if (o[n] > keys.cap) return fail("key offsets run past the keys buffer");
  out->data = keys.addr;
  out->offsets = (const uint64_t *)o;
  return RSK_OK;
}

int rsk_shim_init(int32_t device, int64_t *ctx_out) {
  ENTER();
  rsk_options o;
  memset(&o, 0, sizeof o);
  o.device = device;
  o.redis_version = 320;
  rsk_ctx *c = NULL;
  int rc = rsk_init(&o, &c);
  *ctx_out = rc ? 0 : (int64_t)(intptr_t)c;
  return rc;
}

int rsk_shim_shutdown(int64_t ctx) {
  ENTER();
  return rsk_shutdown((rsk_ctx *)(intptr_t)ctx);
}

int rsk_shim_hll_create(int64_t ctx, int64_t n_sketches, int64_t *hll_out) {
  ENTER();
  if (n_sketches <= 0) return fail("a pool needs at least one sketch");
  rsk_hll *h = NULL;
  int rc = rsk_hll_create((rsk_ctx *)(intptr_t)ctx, (uint64_t)n_sketches, &h);
  *hll_out = rc ? 0 : (int64_t)(intptr_t)h;
  return rc;
}

int rsk_shim_hll_destroy(int64_t hll) {
  ENTER();
  return rsk_hll_destroy((rsk_hll *)(intptr_t)hll);
}

static int check_id(int64_t hll, int64_t id) {
  if (!hll) return fail("sketch handle is null");
  if (id < 0 || (uint64_t)id >= rsk_hll_size((const rsk_hll *)(intptr_t)hll)) return fail("sketch id out of range");
  return RSK_OK;
}

int rsk_shim_hll_add(int64_t hll, int64_t id, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                     uint8_t *changed_out) {
  ENTER();
  rsk_keys k;
  int rc = check_id(hll, id);
  if (!rc) rc = rsk_shim_keys(keys, offsets, n, &k);
  if (rc) return rc;
  return rsk_hll_add((rsk_hll *)(intptr_t)hll, (uint64_t)id, &k, changed_out);
}

int rsk_shim_hll_add_each(int64_t hll, int64_t id, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                          uint8_t *replies, int64_t replies_len) {
  ENTER();
  rsk_keys k;
  int rc = check_id(hll, id);
  if (!rc) rc = rsk_shim_keys(keys, offsets, n, &k);
  if (rc) return rc;
  if (replies_len < n || (n > 0 && !replies)) return fail("reply array shorter than the batch");
  return rsk_hll_add_each((rsk_hll *)(intptr_t)hll, (uint64_t)id, &k, replies);
}

int rsk_shim_hll_count(int64_t hll, int64_t id, int64_t *out) {
  ENTER();
  int rc = check_id(hll, id);
  if (rc) return rc;
  uint64_t ids[1] = {(uint64_t)id}, v[1] = {0};
  rc = rsk_hll_count((rsk_hll *)(intptr_t)hll, ids, 1, v);
  *out = (int64_t)v[0];
  return rc;
}

#define SHIM_MAX_MEMBERS 4096

int rsk_shim_hll_count_union(const int64_t *hlls, const int64_t *ids, int32_t k, int64_t *out) {
  ENTER();
  if (k < 1 || k > SHIM_MAX_MEMBERS) return fail("countWith takes 1..4096 sketches");
  rsk_hll *hs[SHIM_MAX_MEMBERS];
  uint64_t is[SHIM_MAX_MEMBERS];
  for (int32_t i = 0; i < k; ++i) {
    int rc = check_id(hlls[i], ids[i]);
    if (rc) return rc;
    hs[i] = (rsk_hll *)(intptr_t)hlls[i];
    is[i] = (uint64_t)ids[i];
  }
  uint64_t v = 0;
  int rc = rsk_hll_count_union(hs, is, (uint32_t)k, &v);
  *out = (int64_t)v;
  return rc;
}

int rsk_shim_hll_merge(int64_t dst, int64_t dst_id, const int64_t *srcs, const int64_t *src_ids, int32_t k) {
  ENTER();
  if (k < 0 || k > SHIM_MAX_MEMBERS) return fail("mergeWith takes 0..4096 sketches");
  int rc = check_id(dst, dst_id);
  if (rc) return rc;
  rsk_hll *hs[SHIM_MAX_MEMBERS];
  uint64_t is[SHIM_MAX_MEMBERS];
  for (int32_t i = 0; i < k; ++i) {
    rc = check_id(srcs[i], src_ids[i]);
    if (rc) return rc;
    hs[i] = (rsk_hll *)(intptr_t)srcs[i];
    is[i] = (uint64_t)src_ids[i];
  }
  return rsk_hll_merge((rsk_hll *)(intptr_t)dst, (uint64_t)dst_id, hs, is, (uint32_t)k);
}

int rsk_shim_hll_delete(int64_t hll, int64_t id) {
  ENTER();
  int rc = check_id(hll, id);
  return rc ? rc : rsk_hll_delete((rsk_hll *)(intptr_t)hll, (uint64_t)id);
}

int rsk_shim_bloom_params(int64_t expected_insertions, double false_probability, int32_t extended,
                          int64_t *size_out, int32_t *k_out) {
  ENTER();
  return rsk_bloom_params(expected_insertions, false_probability, extended ? RSK_BLOOM_EXTENDED : RSK_BLOOM_COMPAT,
                          size_out, k_out);
}

int rsk_shim_bloom_create(int64_t ctx, int64_t size, int32_t k, int64_t *bloom_out) {
  ENTER();
  rsk_bloom *b = NULL;
  int rc = rsk_bloom_create((rsk_ctx *)(intptr_t)ctx, size, k, &b);
  *bloom_out = rc ? 0 : (int64_t)(intptr_t)b;
  return rc;
}

int rsk_shim_bloom_destroy(int64_t bloom) {
  ENTER();
  return rsk_bloom_destroy((rsk_bloom *)(intptr_t)bloom);
}

int rsk_shim_bloom_add(int64_t bloom, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n, uint8_t *replies,
                       int64_t replies_len) {
  ENTER();
  if (!bloom) return RSK_ERR_NOT_INITIALIZED; /* "Bloom filter is not initialized!" (:217) */
  rsk_keys k;
  int rc = rsk_shim_keys(keys, offsets, n, &k);
  if (rc) return rc;
  if (replies && replies_len < n) return fail("reply array shorter than the batch");
  return rsk_bloom_add((rsk_bloom *)(intptr_t)bloom, &k, replies);
}

int rsk_shim_bloom_contains(int64_t bloom, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n, uint8_t *out,
                            int64_t out_len) {
  ENTER();
  if (!bloom) return RSK_ERR_NOT_INITIALIZED;
  rsk_keys k;
  int rc = rsk_shim_keys(keys, offsets, n, &k);
  if (rc) return rc;
  if (out_len < n || (n > 0 && !out)) return fail("reply array shorter than the batch");
  return rsk_bloom_contains((rsk_bloom *)(intptr_t)bloom, &k, out);
}

int rsk_shim_bloom_count(int64_t bloom, int32_t *out) {
  ENTER();
  if (!bloom) return RSK_ERR_NOT_INITIALIZED;
  return rsk_bloom_count((rsk_bloom *)(intptr_t)bloom, out);
}
