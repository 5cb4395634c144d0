/*
 * rsketch_shim.c -- argument checks, conversions and the name -> object
 * keyspace of the Java binding (see rsketch_shim.h).  Plain C11 + pthreads;
 * links librsketch.so.
 *
 * Locking: the registry mutex guards the map and the reference counts only;
 * no library call is made while it is held (object creation and destruction
 * happen outside it), so a completion callback -- which releases its
 * references under the same mutex -- can never wait on a thread that waits on
 * the device.  Objects whose last reference drops inside a callback (where no
 * library call is allowed) are destroyed by the next call into the space.
 */
#include "rsketch_shim.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static _Thread_local char shim_err[256];
static _Thread_local int shim_failed;

static int fail_code(int code, const char *msg) {
  snprintf(shim_err, sizeof shim_err, "%s", msg);
  shim_failed = 1;
  return code;
}
static int fail(const char *msg) { return fail_code(RSK_ERR_INVALID_ARG, msg); }

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
    default: /* WRONGTYPE, INVALID_HLL, DEVICE, NO_DEVICE, RSK_SHIM_CONFIG_CHANGED, RSK_SHIM_REDIS_ERROR */
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

/* ------------------------------------------------------------ keyspace */
typedef struct entry {
  char *name;
  uint64_t hash;
  int32_t type; /* RSK_SHIM_HLL / RSK_SHIM_BLOOM / RSK_SHIM_BITSET */
  rsk_hll *hll; /* a one-sketch pool */
  rsk_bloom *bloom;
  /* RSK_SHIM_BITSET: the string; RSK_SHIM_BLOOM: the view of the filter's
   * bits (rsk_bloom_bitset), made on the first RBitSet call on the name */
  rsk_bitset *bits;
  rsk_shim_bloom_config cfg;
  int refs; /* the map's reference + calls in flight */
  struct entry *next;
} entry;

typedef struct rsk_shim_space {
  rsk_ctx *ctx;
  int32_t extended;
  pthread_mutex_t mu;
  entry **buckets;
  size_t nbuckets, count;
  entry *grave; /* unreferenced entries to destroy (their last release ran in a callback) */
} space;

static uint64_t name_hash(const char *s) { /* FNV-1a */
  uint64_t h = 1469598103934665603ull;
  for (; *s; ++s) h = (h ^ (unsigned char)*s) * 1099511628211ull;
  return h;
}

static void destroy_entry(entry *e) {
  if (e->hll) (void)rsk_hll_destroy(e->hll);
  if (e->bits) (void)rsk_bitset_destroy(e->bits); /* a view goes before its filter */
  if (e->bloom) (void)rsk_bloom_destroy(e->bloom);
  free(e->name);
  free(e);
}

/* Destroys what callbacks left behind (never under the mutex). */
static void drain(space *s) {
  pthread_mutex_lock(&s->mu);
  entry *g = s->grave;
  s->grave = NULL;
  pthread_mutex_unlock(&s->mu);
  while (g) {
    entry *nx = g->next;
    destroy_entry(g);
    g = nx;
  }
}

static entry **slot_of(space *s, const char *name, uint64_t h) {
  entry **p = &s->buckets[h & (s->nbuckets - 1)];
  while (*p && ((*p)->hash != h || strcmp((*p)->name, name) != 0)) p = &(*p)->next;
  return p;
}

static void grow(space *s) { /* under the mutex */
  if (s->count < s->nbuckets) return;
  const size_t nb = s->nbuckets * 2;
  entry **b = calloc(nb, sizeof *b);
  if (!b) return; /* keep the longer chains */
  for (size_t i = 0; i < s->nbuckets; ++i) {
    entry *e = s->buckets[i];
    while (e) {
      entry *nx = e->next;
      e->next = b[e->hash & (nb - 1)];
      b[e->hash & (nb - 1)] = e;
      e = nx;
    }
  }
  free(s->buckets);
  s->buckets = b;
  s->nbuckets = nb;
}

/* The entry of `name` with one more reference (NULL if absent). */
static entry *acquire(space *s, const char *name) {
  const uint64_t h = name_hash(name);
  pthread_mutex_lock(&s->mu);
  entry *e = *slot_of(s, name, h);
  if (e) ++e->refs;
  pthread_mutex_unlock(&s->mu);
  return e;
}

static void release_ex(space *s, entry *e, int in_callback) {
  if (!e) return;
  pthread_mutex_lock(&s->mu);
  const int last = --e->refs == 0;
  if (last && in_callback) {
    e->next = s->grave;
    s->grave = e;
  }
  pthread_mutex_unlock(&s->mu);
  if (last && !in_callback) destroy_entry(e);
}
static void release(space *s, entry *e) { release_ex(s, e, 0); }

/* Inserts a fresh entry unless the name exists meanwhile; returns the entry
 * in force (referenced) and sets *inserted.  fresh is consumed. */
static entry *insert_or_get(space *s, entry *fresh, int *inserted) {
  pthread_mutex_lock(&s->mu);
  entry **p = slot_of(s, fresh->name, fresh->hash);
  entry *e = *p;
  if (e) {
    ++e->refs;
    *inserted = 0;
  } else {
    fresh->refs = 2; /* the map's + the caller's */
    fresh->next = NULL;
    *p = fresh;
    ++s->count;
    grow(s);
    e = fresh;
    *inserted = 1;
  }
  pthread_mutex_unlock(&s->mu);
  if (!*inserted) destroy_entry(fresh);
  return e;
}

static entry *new_entry(const char *name, int32_t type) {
  entry *e = calloc(1, sizeof *e);
  if (!e) return NULL;
  e->name = strdup(name);
  if (!e->name) {
    free(e);
    return NULL;
  }
  e->hash = name_hash(name);
  e->type = type;
  return e;
}

static space *sp(int64_t h) { return (space *)(intptr_t)h; }

/* An HLL key of `name` (created when missing if `create`), referenced. */
static int hll_entry(space *s, const char *name, int create, entry **out) {
  *out = NULL;
  if (!name) return fail("name is null");
  entry *e = acquire(s, name);
  if (e) {
    if (e->type != RSK_SHIM_HLL) {
      release(s, e);
      return fail_code(RSK_ERR_WRONGTYPE, "WRONGTYPE Key is not a valid HyperLogLog string value.");
    }
    *out = e;
    return RSK_OK;
  }
  if (!create) return RSK_OK;
  entry *f = new_entry(name, RSK_SHIM_HLL);
  if (!f) return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  int rc = rsk_hll_create(s->ctx, 1, &f->hll);
  if (rc) {
    free(f->name);
    free(f);
    return rc;
  }
  int ins = 0;
  e = insert_or_get(s, f, &ins);
  if (e->type != RSK_SHIM_HLL) {
    release(s, e);
    return fail_code(RSK_ERR_WRONGTYPE, "WRONGTYPE Key is not a valid HyperLogLog string value.");
  }
  *out = e;
  return RSK_OK;
}

/* The Bloom filter of `name`, referenced; NOT_INITIALIZED when absent. */
static int bloom_entry(space *s, const char *name, entry **out) {
  *out = NULL;
  if (!name) return fail("name is null");
  entry *e = acquire(s, name);
  if (!e) return fail_code(RSK_ERR_NOT_INITIALIZED, "Bloom filter is not initialized!");
  if (e->type != RSK_SHIM_BLOOM) {
    release(s, e);
    return fail_code(RSK_ERR_WRONGTYPE, "WRONGTYPE Operation against a key holding the wrong kind of value");
  }
  *out = e;
  return RSK_OK;
}

int rsk_shim_init(int32_t device, int32_t extended_bloom, int64_t *space_out) {
  ENTER();
  if (!space_out) return fail("space_out is null");
  *space_out = 0;
  space *s = calloc(1, sizeof *s);
  if (!s) return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  s->nbuckets = 64;
  s->buckets = calloc(s->nbuckets, sizeof *s->buckets);
  if (!s->buckets) {
    free(s);
    return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  if (rsk_abi_version() != RSK_ABI_VERSION) {
    free(s->buckets);
    free(s);
    return fail_code(RSK_ERR_NO_DEVICE, "librsketch.so was built against another rsketch.h (RSK_ABI_VERSION)");
  }
  rsk_options o;
  memset(&o, 0, sizeof o);
  o.device = device;
  o.redis_version = 320;
  int rc = rsk_init(&o, &s->ctx);
  if (rc) {
    free(s->buckets);
    free(s);
    return rc;
  }
  pthread_mutex_init(&s->mu, NULL);
  s->extended = extended_bloom ? 1 : 0;
  *space_out = (int64_t)(intptr_t)s;
  return RSK_OK;
}

int rsk_shim_shutdown(int64_t h) {
  ENTER();
  space *s = sp(h);
  if (!s) return RSK_OK;
  (void)rsk_sync(s->ctx); /* every completion has run */
  drain(s);
  for (size_t i = 0; i < s->nbuckets; ++i) {
    entry *e = s->buckets[i];
    while (e) {
      entry *nx = e->next;
      destroy_entry(e);
      e = nx;
    }
  }
  free(s->buckets);
  pthread_mutex_destroy(&s->mu);
  const int rc = rsk_shutdown(s->ctx);
  free(s);
  return rc;
}

rsk_ctx *rsk_shim_context(int64_t h) {
  space *s = sp(h);
  return s ? s->ctx : NULL;
}

int rsk_shim_sync(int64_t h) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  const int rc = rsk_sync(s->ctx); /* every call issued so far has completed and its callback returned */
  drain(s);
  return rc;
}

int rsk_shim_lookup(int64_t h, const char *name, int32_t *type_out, int64_t *handle_out) {
  ENTER();
  space *s = sp(h);
  if (!s || !name || !type_out || !handle_out) return fail("null argument");
  drain(s);
  entry *e = acquire(s, name);
  *type_out = e ? e->type : RSK_SHIM_NONE;
  *handle_out = e ? (int64_t)(intptr_t)(e->hll ? (void *)e->hll : e->bloom ? (void *)e->bloom : (void *)e->bits) : 0;
  release(s, e);
  return RSK_OK;
}

int rsk_shim_delete(int64_t h, const char *name, int32_t *deleted_out) {
  ENTER();
  space *s = sp(h);
  if (!s || !name) return fail("null argument");
  drain(s);
  const uint64_t hh = name_hash(name);
  pthread_mutex_lock(&s->mu);
  entry **p = slot_of(s, name, hh);
  entry *e = *p;
  if (e) {
    *p = e->next;
    --s->count;
  }
  pthread_mutex_unlock(&s->mu);
  if (deleted_out) *deleted_out = e ? 1 : 0;
  release(s, e); /* the map's reference: destroyed now or after the last call on it */
  return RSK_OK;
}

int rsk_shim_rename(int64_t h, const char *old_name, const char *new_name, int32_t nx, int32_t *renamed_out) {
  ENTER();
  space *s = sp(h);
  if (!s || !old_name || !new_name) return fail("null argument");
  drain(s);
  if (renamed_out) *renamed_out = 0;
  char *nn = strdup(new_name);
  if (!nn) return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  entry *victim = NULL;
  int rc = RSK_OK;
  pthread_mutex_lock(&s->mu);
  entry **po = slot_of(s, old_name, name_hash(old_name));
  entry *e = *po;
  if (!e) {
    rc = fail("ERR no such key");
  } else if (strcmp(old_name, new_name) != 0) {
    entry **pn = slot_of(s, new_name, name_hash(new_name));
    if (*pn && nx) {
      rc = RSK_OK; /* RENAMENX onto an existing key: 0 */
    } else {
      if (*pn) { /* RENAME replaces the target */
        victim = *pn;
        *pn = victim->next;
        --s->count;
      }
      po = slot_of(s, old_name, name_hash(old_name)); /* the chain may have changed */
      *po = e->next;
      free(e->name);
      e->name = nn;
      nn = NULL;
      e->hash = name_hash(e->name);
      entry **dst = slot_of(s, e->name, e->hash);
      e->next = NULL;
      *dst = e;
      if (renamed_out) *renamed_out = 1;
    }
  } else if (renamed_out) {
    *renamed_out = nx ? 0 : 1;
  }
  pthread_mutex_unlock(&s->mu);
  free(nn);
  release(s, victim); /* the map's reference of the replaced object */
  return rc;
}

/* --------------------------------------------------------------- HLL */
int rsk_shim_hll_add(int64_t h, const char *name, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                     uint8_t *changed_out) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  rsk_keys k;
  int rc = rsk_shim_keys(keys, offsets, n, &k);
  if (rc) return rc;
  entry *e;
  if ((rc = hll_entry(s, name, 1, &e))) return rc;
  rc = rsk_hll_add(e->hll, 0, &k, changed_out);
  release(s, e);
  return rc;
}

int rsk_shim_hll_add_each(int64_t h, const char *name, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                          uint8_t *replies, int64_t replies_len) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  rsk_keys k;
  int rc = rsk_shim_keys(keys, offsets, n, &k);
  if (rc) return rc;
  if (replies_len < n || (n > 0 && !replies)) return fail("reply array shorter than the batch");
  entry *e;
  if ((rc = hll_entry(s, name, 1, &e))) return rc;
  rc = rsk_hll_add_each(e->hll, 0, &k, replies);
  release(s, e);
  return rc;
}

int rsk_shim_hll_count(int64_t h, const char *name, int64_t *out) {
  ENTER();
  space *s = sp(h);
  if (!s || !out) return fail("null argument");
  drain(s);
  entry *e;
  int rc = hll_entry(s, name, 0, &e);
  if (rc) return rc;
  *out = 0;
  if (!e) return RSK_OK; /* PFCOUNT of a missing key: 0, nothing created */
  uint64_t id = 0, v = 0;
  rc = rsk_hll_count(e->hll, &id, 1, &v);
  *out = (int64_t)v;
  release(s, e);
  return rc;
}

#define SHIM_MAX_MEMBERS 4096

/* The existing members of names[0..k) (missing ones skipped), referenced. */
static int members(space *s, const char *const *names, int32_t k, entry **es, int32_t *m) {
  *m = 0;
  if (k < 0 || k > SHIM_MAX_MEMBERS) return fail("at most 4096 keys per call");
  if (k > 0 && !names) return fail("names is null");
  for (int32_t i = 0; i < k; ++i) {
    entry *e;
    int rc = hll_entry(s, names[i], 0, &e);
    if (rc) {
      for (int32_t j = 0; j < *m; ++j) release(s, es[j]);
      *m = 0;
      return rc;
    }
    if (e) es[(*m)++] = e;
  }
  return RSK_OK;
}

int rsk_shim_hll_count_with(int64_t h, const char *const *names, int32_t k, int64_t *out) {
  ENTER();
  space *s = sp(h);
  if (!s || !out) return fail("null argument");
  if (k < 1 || !names) return fail("countWith takes at least one key");
  if (k == 1) return rsk_shim_hll_count(h, names[0], out); /* PFCOUNT of one key: the cached path */
  drain(s);
  entry *es[SHIM_MAX_MEMBERS];
  int32_t m;
  int rc = members(s, names, k, es, &m);
  if (rc) return rc;
  *out = 0;
  if (m > 0) { /* multi-key PFCOUNT: union in raw order, no cache */
    rsk_hll *hs[SHIM_MAX_MEMBERS];
    uint64_t ids[SHIM_MAX_MEMBERS];
    for (int32_t i = 0; i < m; ++i) {
      hs[i] = es[i]->hll;
      ids[i] = 0;
    }
    uint64_t v = 0;
    rc = rsk_hll_count_union(hs, ids, (uint32_t)m, &v);
    *out = (int64_t)v;
  }
  for (int32_t i = 0; i < m; ++i) release(s, es[i]);
  return rc;
}

int rsk_shim_hll_merge_with(int64_t h, const char *dst, const char *const *srcs, int32_t k) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  entry *es[SHIM_MAX_MEMBERS];
  int32_t m;
  int rc = members(s, srcs, k, es, &m);
  if (rc) return rc;
  entry *d;
  if ((rc = hll_entry(s, dst, 1, &d))) {
    for (int32_t i = 0; i < m; ++i) release(s, es[i]);
    return rc;
  }
  rsk_hll *hs[SHIM_MAX_MEMBERS];
  uint64_t ids[SHIM_MAX_MEMBERS];
  for (int32_t i = 0; i < m; ++i) {
    hs[i] = es[i]->hll;
    ids[i] = 0;
  }
  rc = rsk_hll_merge(d->hll, 0, hs, ids, (uint32_t)m);
  release(s, d);
  for (int32_t i = 0; i < m; ++i) release(s, es[i]);
  return rc;
}

int rsk_shim_batch_hll_add(int64_t h, const char *const *names, int32_t n_names, const int32_t *name_of,
                           rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n, uint8_t *replies, int64_t replies_len) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  rsk_keys k;
  int rc = rsk_shim_keys(keys, offsets, n, &k);
  if (rc) return rc;
  if (n > 0 && (!names || !name_of || n_names < 1)) return fail("names is null");
  if (replies_len < n || (n > 0 && !replies)) return fail("reply array shorter than the batch");
  for (int64_t i = 0; i < n; ++i)
    if (name_of[i] < 0 || name_of[i] >= n_names) return fail("element refers to no name of the batch");
  const int64_t *o = (const int64_t *)offsets.addr;
  const uint8_t *data = (const uint8_t *)keys.addr;
  /* elements grouped by name, input order kept inside a name (a stable
   * counting sort), each name's keys gathered into one batch */
  int64_t *start = calloc((size_t)n_names + 1, sizeof(int64_t));
  int64_t *idx = malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int64_t *goff = malloc(sizeof(int64_t) * (size_t)(n + 1));
  uint8_t *gbytes = malloc((size_t)(n > 0 ? o[n] - o[0] : 0) + 1);
  uint8_t *grep = malloc((size_t)(n > 0 ? n : 1));
  if (!start || !idx || !goff || !gbytes || !grep) {
    free(start), free(idx), free(goff), free(gbytes), free(grep);
    return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  for (int64_t i = 0; i < n; ++i) ++start[name_of[i] + 1];
  for (int32_t j = 0; j < n_names; ++j) start[j + 1] += start[j];
  {
    int64_t *fill = malloc(sizeof(int64_t) * (size_t)n_names);
    if (!fill) {
      free(start), free(idx), free(goff), free(gbytes), free(grep);
      return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
    }
    memcpy(fill, start, sizeof(int64_t) * (size_t)n_names);
    for (int64_t i = 0; i < n; ++i) idx[fill[name_of[i]]++] = i;
    free(fill);
  }
  for (int32_t j = 0; j < n_names && rc == RSK_OK; ++j) {
    const int64_t m = start[j + 1] - start[j];
    if (m == 0) continue;
    const int64_t *ix = idx + start[j];
    int64_t pos = 0;
    goff[0] = 0;
    for (int64_t q = 0; q < m; ++q) {
      const int64_t i = ix[q], len = o[i + 1] - o[i];
      memcpy(gbytes + pos, data + o[i], (size_t)len);
      pos += len;
      goff[q + 1] = pos;
    }
    const rsk_keys gk = {gbytes, (const uint64_t *)goff, (uint64_t)m, 0, RSK_MEM_HOST};
    entry *e;
    if ((rc = hll_entry(s, names[j], 1, &e))) break;
    rc = rsk_hll_add_each(e->hll, 0, &gk, grep);
    release(s, e);
    for (int64_t q = 0; q < m && rc == RSK_OK; ++q) replies[ix[q]] = grep[q];
  }
  free(start);
  free(idx), free(goff), free(gbytes), free(grep);
  return rc;
}

/* ----------------------------------------------------------- async */
typedef struct shim_async {
  space *s;
  rsk_done_fn cb;
  void *user;
  int32_t m;
  entry *es[]; /* released when the call completes */
} shim_async;

static shim_async *async_new(space *s, rsk_done_fn cb, void *user, int32_t cap) {
  shim_async *a = malloc(sizeof *a + sizeof(entry *) * (size_t)(cap > 0 ? cap : 1));
  if (!a) return NULL;
  a->s = s;
  a->cb = cb;
  a->user = user;
  a->m = 0;
  return a;
}

static void async_done(void *p, int status, uint64_t value) { /* completion thread: no library call */
  shim_async *a = p;
  for (int32_t i = 0; i < a->m; ++i) release_ex(a->s, a->es[i], 1);
  if (a->cb) a->cb(a->user, status, value);
  free(a);
}

/* A call the library refused: it never fires, so the references go now. */
static int async_refused(shim_async *a, int rc) {
  for (int32_t i = 0; i < a->m; ++i) release(a->s, a->es[i]);
  free(a);
  return rc;
}

int rsk_shim_hll_add_async(int64_t h, const char *name, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                           rsk_done_fn cb, void *user) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  rsk_keys k;
  int rc = rsk_shim_keys(keys, offsets, n, &k);
  if (rc) return rc;
  entry *e;
  if ((rc = hll_entry(s, name, 1, &e))) return rc;
  shim_async *a = async_new(s, cb, user, 1);
  if (!a) {
    release(s, e);
    return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  a->es[a->m++] = e;
  rc = rsk_hll_add_async(e->hll, 0, &k, async_done, a);
  return rc ? async_refused(a, rc) : RSK_OK;
}

int rsk_shim_hll_count_async(int64_t h, const char *name, rsk_done_fn cb, void *user) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  entry *e;
  int rc = hll_entry(s, name, 0, &e);
  if (rc) return rc;
  if (!e) { /* missing key: 0, nothing to wait for */
    if (cb) cb(user, RSK_OK, 0);
    return RSK_OK;
  }
  shim_async *a = async_new(s, cb, user, 1);
  if (!a) {
    release(s, e);
    return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  a->es[a->m++] = e;
  rc = rsk_hll_count_async(e->hll, 0, async_done, a);
  return rc ? async_refused(a, rc) : RSK_OK;
}

int rsk_shim_hll_count_with_async(int64_t h, const char *const *names, int32_t k, rsk_done_fn cb, void *user) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  if (k < 1 || !names) return fail("countWith takes at least one key");
  if (k == 1) return rsk_shim_hll_count_async(h, names[0], cb, user);
  drain(s);
  shim_async *a = async_new(s, cb, user, k);
  if (!a) return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  int rc = members(s, names, k, a->es, &a->m);
  if (rc) {
    free(a);
    return rc;
  }
  if (a->m == 0) {
    free(a);
    if (cb) cb(user, RSK_OK, 0);
    return RSK_OK;
  }
  rsk_hll *hs[SHIM_MAX_MEMBERS];
  uint64_t ids[SHIM_MAX_MEMBERS];
  for (int32_t i = 0; i < a->m; ++i) {
    hs[i] = a->es[i]->hll;
    ids[i] = 0;
  }
  rc = rsk_hll_count_union_async(hs, ids, (uint32_t)a->m, async_done, a);
  return rc ? async_refused(a, rc) : RSK_OK;
}

int rsk_shim_hll_merge_with_async(int64_t h, const char *dst, const char *const *srcs, int32_t k, rsk_done_fn cb,
                                  void *user) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  shim_async *a = async_new(s, cb, user, k + 1);
  if (!a) return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  int rc = members(s, srcs, k, a->es, &a->m);
  if (rc) {
    free(a);
    return rc;
  }
  entry *d;
  if ((rc = hll_entry(s, dst, 1, &d))) return async_refused(a, rc);
  rsk_hll *hs[SHIM_MAX_MEMBERS];
  uint64_t ids[SHIM_MAX_MEMBERS];
  const int32_t m = a->m;
  for (int32_t i = 0; i < m; ++i) {
    hs[i] = a->es[i]->hll;
    ids[i] = 0;
  }
  a->es[a->m++] = d;
  rc = rsk_hll_merge_async(d->hll, 0, hs, ids, (uint32_t)m, async_done, a);
  return rc ? async_refused(a, rc) : RSK_OK;
}

/* ------------------------------------------------------------- Bloom */
int rsk_shim_bloom_try_init(int64_t h, const char *name, int64_t expected_insertions, double false_probability,
                            int32_t *created_out, rsk_shim_bloom_config *cfg_out) {
  ENTER();
  space *s = sp(h);
  if (!s || !name || !created_out) return fail("null argument");
  drain(s);
  *created_out = 0;
  int64_t size = 0;
  int32_t k = 0;
  /* optimalNumOfBits / MAX_SIZE first: the reference throws before asking Redis (:224-228) */
  int rc = rsk_bloom_params(expected_insertions, false_probability,
                            s->extended ? RSK_BLOOM_EXTENDED : RSK_BLOOM_COMPAT, &size, &k);
  if (rc) return rc;
  entry *e = acquire(s, name);
  if (!e) {
    entry *f = new_entry(name, RSK_SHIM_BLOOM);
    if (!f) return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
    if ((rc = rsk_bloom_create(s->ctx, size, k, &f->bloom))) {
      free(f->name);
      free(f);
      return rc;
    }
    f->cfg.size = size;
    f->cfg.hash_iterations = k;
    f->cfg.expected_insertions = expected_insertions;
    f->cfg.false_probability = false_probability;
    int ins = 0;
    e = insert_or_get(s, f, &ins);
    *created_out = ins;
  }
  if (e->type != RSK_SHIM_BLOOM) {
    release(s, e);
    *created_out = 0;
    return fail_code(RSK_ERR_WRONGTYPE, "WRONGTYPE Operation against a key holding the wrong kind of value");
  }
  if (cfg_out) *cfg_out = e->cfg;
  release(s, e);
  return RSK_OK;
}

int rsk_shim_bloom_get_config(int64_t h, const char *name, rsk_shim_bloom_config *out) {
  ENTER();
  space *s = sp(h);
  if (!s || !out) return fail("null argument");
  drain(s);
  entry *e;
  int rc = bloom_entry(s, name, &e);
  if (rc) return rc;
  *out = e->cfg;
  release(s, e);
  return RSK_OK;
}

/* The referenced filter of `name` if the caller's (size, k) is still its config. */
static int bloom_checked(space *s, const char *name, int64_t size, int32_t k, entry **out) {
  int rc = bloom_entry(s, name, out);
  if (rc) return rc;
  if ((*out)->cfg.size != size || (*out)->cfg.hash_iterations != k) {
    release(s, *out);
    *out = NULL;
    return fail_code(RSK_SHIM_CONFIG_CHANGED, "Bloom filter config has been changed");
  }
  return RSK_OK;
}

int rsk_shim_bloom_add(int64_t h, const char *name, int64_t size, int32_t k, rsk_shim_buf keys, rsk_shim_buf offsets,
                       int64_t n, uint8_t *replies, int64_t replies_len) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  entry *e;
  int rc = bloom_checked(s, name, size, k, &e);
  if (rc) return rc;
  rsk_keys kk;
  if (!(rc = rsk_shim_keys(keys, offsets, n, &kk))) {
    if (replies && replies_len < n) rc = fail("reply array shorter than the batch");
    else rc = rsk_bloom_add(e->bloom, &kk, replies);
  }
  release(s, e);
  return rc;
}

int rsk_shim_bloom_contains(int64_t h, const char *name, int64_t size, int32_t k, rsk_shim_buf keys,
                            rsk_shim_buf offsets, int64_t n, uint8_t *out, int64_t out_len) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  entry *e;
  int rc = bloom_checked(s, name, size, k, &e);
  if (rc) return rc;
  rsk_keys kk;
  if (!(rc = rsk_shim_keys(keys, offsets, n, &kk))) {
    if (out_len < n || (n > 0 && !out)) rc = fail("reply array shorter than the batch");
    else rc = rsk_bloom_contains(e->bloom, &kk, out);
  }
  release(s, e);
  return rc;
}

int rsk_shim_bloom_count(int64_t h, const char *name, int32_t *out) {
  ENTER();
  space *s = sp(h);
  if (!s || !out) return fail("null argument");
  drain(s);
  entry *e;
  int rc = bloom_entry(s, name, &e);
  if (rc) return rc;
  rc = rsk_bloom_count(e->bloom, out);
  release(s, e);
  return rc;
}

int rsk_shim_bloom_add_async(int64_t h, const char *name, int64_t size, int32_t k, rsk_shim_buf keys,
                             rsk_shim_buf offsets, int64_t n, uint8_t *replies, int64_t replies_len, rsk_done_fn cb,
                             void *user) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  rsk_keys kk;
  int rc = rsk_shim_keys(keys, offsets, n, &kk);
  if (rc) return rc;
  if (replies && replies_len < n) return fail("reply array shorter than the batch");
  entry *e;
  if ((rc = bloom_checked(s, name, size, k, &e))) return rc;
  shim_async *a = async_new(s, cb, user, 1);
  if (!a) {
    release(s, e);
    return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  a->es[a->m++] = e;
  rc = rsk_bloom_add_async(e->bloom, &kk, replies, async_done, a);
  return rc ? async_refused(a, rc) : RSK_OK;
}

int rsk_shim_bloom_contains_async(int64_t h, const char *name, int64_t size, int32_t k, rsk_shim_buf keys,
                                  rsk_shim_buf offsets, int64_t n, uint8_t *out, int64_t out_len, rsk_done_fn cb,
                                  void *user) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  rsk_keys kk;
  int rc = rsk_shim_keys(keys, offsets, n, &kk);
  if (rc) return rc;
  if (out_len < n || (n > 0 && !out)) return fail("reply array shorter than the batch");
  entry *e;
  if ((rc = bloom_checked(s, name, size, k, &e))) return rc;
  shim_async *a = async_new(s, cb, user, 1);
  if (!a) {
    release(s, e);
    return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  a->es[a->m++] = e;
  rc = rsk_bloom_contains_async(e->bloom, &kk, out, async_done, a);
  return rc ? async_refused(a, rc) : RSK_OK;
}

/* ------------------------------------------------------------ RBitSet */
#define RSK_BITOFF_MAX 4294967295LL /* Redis: a string holds at most 512 MB */

static int redis_err(const char *msg) { return fail_code(RSK_SHIM_REDIS_ERROR, msg); }

/* The string of `name` as an rsk_bitset, referenced: a plain RBitSet string,
 * or the bits of a Bloom filter (the view, made once per filter).  *bits_out
 * NULL (and *e_out NULL) when the name is absent and !create; an HLL is
 * refused with WRONGTYPE (its Redis string is not exposed bit-wise here). */
static int bits_entry(space *s, const char *name, int create, entry **e_out, rsk_bitset **bits_out) {
  *e_out = NULL;
  *bits_out = NULL;
  if (!name) return fail("name is null");
  entry *e = acquire(s, name);
  if (!e) {
    if (!create) return RSK_OK;
    entry *f = new_entry(name, RSK_SHIM_BITSET);
    if (!f) return fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
    int rc = rsk_bitset_create(s->ctx, &f->bits);
    if (rc) {
      free(f->name);
      free(f);
      return rc;
    }
    int ins = 0;
    e = insert_or_get(s, f, &ins);
  }
  if (e->type == RSK_SHIM_HLL) {
    release(s, e);
    return fail_code(RSK_ERR_WRONGTYPE,
                     "WRONGTYPE the key holds a GPU HyperLogLog; its Redis string is not exposed as an RBitSet");
  }
  if (e->type == RSK_SHIM_BLOOM) {
    pthread_mutex_lock(&s->mu);
    rsk_bitset *v = e->bits;
    pthread_mutex_unlock(&s->mu);
    if (!v) { /* made outside the mutex (a library call); the first one made wins */
      int rc = rsk_bloom_bitset(e->bloom, &v);
      if (rc) {
        release(s, e);
        return rc;
      }
      pthread_mutex_lock(&s->mu);
      rsk_bitset *won = e->bits;
      if (!won) e->bits = v;
      pthread_mutex_unlock(&s->mu);
      if (won) {
        (void)rsk_bitset_destroy(v);
        v = won;
      }
    }
    *bits_out = v;
  } else {
    *bits_out = e->bits;
  }
  *e_out = e;
  return RSK_OK;
}

static int offsets_ok(const int64_t *offs, int64_t n) {
  if (n < 0) return fail("negative element count");
  if (n > 0 && !offs) return fail("offsets is null");
  for (int64_t i = 0; i < n; ++i)
    if (offs[i] < 0 || offs[i] > RSK_BITOFF_MAX) return redis_err("ERR bit offset is not an integer or out of range");
  return RSK_OK;
}

int rsk_shim_bitset_strlen(int64_t h, const char *name, int64_t *out) {
  ENTER();
  space *s = sp(h);
  if (!s || !out) return fail("null argument");
  drain(s);
  entry *e;
  rsk_bitset *b;
  *out = 0;
  int rc = bits_entry(s, name, 0, &e, &b);
  if (rc || !e) return rc;
  uint64_t v = 0;
  rc = rsk_bitset_strlen(b, &v);
  *out = (int64_t)v;
  release(s, e);
  return rc;
}

int rsk_shim_bitset_get_bytes(int64_t h, const char *name, uint8_t **bytes_out, int64_t *len_out) {
  ENTER();
  space *s = sp(h);
  if (!s || !bytes_out || !len_out) return fail("null argument");
  drain(s);
  *bytes_out = NULL;
  *len_out = -1; /* GET of a missing key: nil */
  entry *e;
  rsk_bitset *b;
  int rc = bits_entry(s, name, 0, &e, &b);
  if (rc || !e) return rc;
  for (;;) { /* another thread may grow the string between STRLEN and GET: size again */
    uint64_t n = 0;
    if ((rc = rsk_bitset_strlen(b, &n))) break;
    uint8_t *buf = malloc((size_t)n + 1);
    if (!buf) {
      rc = fail_code(RSK_ERR_OUT_OF_MEMORY, "host allocation failed");
      break;
    }
    size_t got = 0;
    rc = rsk_bitset_get_bytes(b, buf, (size_t)n + 1, &got);
    if (rc == RSK_ERR_INVALID_ARG) { /* grew meanwhile */
      free(buf);
      continue;
    }
    if (rc) {
      free(buf);
      break;
    }
    if (got == 0) { /* no string: a filter nothing was added to yet, or an emptied string (Redis deletes it) */
      free(buf);
      break;
    }
    *bytes_out = buf;
    *len_out = (int64_t)got;
    break;
  }
  release(s, e);
  return rc;
}

void rsk_shim_free(void *p) { free(p); }

int rsk_shim_bitset_getbits(int64_t h, const char *name, const int64_t *offs, int64_t n, uint8_t *out,
                            int64_t out_len) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  int rc = offsets_ok(offs, n);
  if (rc) return rc;
  if (out_len < n || (n > 0 && !out)) return fail("reply array shorter than the batch");
  entry *e;
  rsk_bitset *b;
  if ((rc = bits_entry(s, name, 0, &e, &b))) return rc;
  if (!e) { /* GETBIT of a missing key: 0 */
    if (n) memset(out, 0, (size_t)n);
    return RSK_OK;
  }
  rc = rsk_bitset_getbits(b, (const uint64_t *)offs, (uint64_t)n, RSK_MEM_HOST, out);
  release(s, e);
  return rc;
}

int rsk_shim_bitset_setbits(int64_t h, const char *name, const int64_t *offs, int64_t n, int32_t value) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  int rc = offsets_ok(offs, n);
  if (rc) return rc;
  if (n == 0) return RSK_OK;
  entry *e;
  rsk_bitset *b;
  if ((rc = bits_entry(s, name, 1, &e, &b))) return rc;
  rc = rsk_bitset_setbits(b, (const uint64_t *)offs, (uint64_t)n, value ? 1 : 0, RSK_MEM_HOST);
  release(s, e);
  return rc;
}

int rsk_shim_bitset_set_range(int64_t h, const char *name, int64_t from, int64_t to, int32_t value) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  if (to <= from) return RSK_OK; /* the reference's loop issues no SETBIT */
  if (from < 0 || to - 1 > RSK_BITOFF_MAX) return redis_err("ERR bit offset is not an integer or out of range");
  entry *e;
  rsk_bitset *b;
  int rc = bits_entry(s, name, 1, &e, &b);
  if (rc) return rc;
  rc = rsk_bitset_set_range(b, (uint64_t)from, (uint64_t)to, value ? 1 : 0);
  release(s, e);
  return rc;
}

int rsk_shim_bitset_cardinality(int64_t h, const char *name, int64_t *out) {
  ENTER();
  space *s = sp(h);
  if (!s || !out) return fail("null argument");
  drain(s);
  *out = 0;
  entry *e;
  rsk_bitset *b;
  int rc = bits_entry(s, name, 0, &e, &b);
  if (rc || !e) return rc;
  uint64_t v = 0;
  rc = rsk_bitset_bitcount(b, &v);
  *out = (int64_t)v;
  release(s, e);
  return rc;
}

int rsk_shim_bitset_length(int64_t h, const char *name, int64_t *out) {
  ENTER();
  space *s = sp(h);
  if (!s || !out) return fail("null argument");
  drain(s);
  *out = 0;
  entry *e;
  rsk_bitset *b;
  int rc = bits_entry(s, name, 0, &e, &b);
  if (rc || !e) return rc;
  uint64_t v = 0;
  rc = rsk_bitset_length(b, &v);
  *out = (int64_t)v;
  release(s, e);
  return rc;
}

int rsk_shim_bitset_set_bytes(int64_t h, const char *name, const uint8_t *bytes, int64_t len) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  if (len < 0 || (len > 0 && !bytes)) return fail("bad byte array");
  if (len > (RSK_BITOFF_MAX >> 3) + 1) return redis_err("ERR string exceeds maximum allowed size (512MB)");
  entry *e;
  rsk_bitset *b;
  int rc = bits_entry(s, name, 1, &e, &b);
  if (rc) return rc;
  rc = rsk_bitset_set_bytes(b, bytes, (size_t)len);
  release(s, e);
  return rc;
}

/* Removes a plain string's entry if it is (still) empty: Redis holds no key
 * for an empty result (BITOP of empty sources, DEL). */
static void drop_if_empty(space *s, const char *name) {
  entry *e = acquire(s, name);
  if (!e) return;
  uint64_t n = 1;
  if (e->type == RSK_SHIM_BITSET && rsk_bitset_strlen(e->bits, &n) == RSK_OK && n == 0) {
    pthread_mutex_lock(&s->mu);
    entry **p = slot_of(s, name, e->hash);
    const int mine = *p == e;
    if (mine) {
      *p = e->next;
      --s->count;
    }
    pthread_mutex_unlock(&s->mu);
    if (mine) release(s, e); /* the map's reference */
  }
  release(s, e);
}

int rsk_shim_bitset_clear(int64_t h, const char *name, int32_t *deleted_out) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  if (deleted_out) *deleted_out = 0;
  entry *e;
  rsk_bitset *b;
  int rc = bits_entry(s, name, 0, &e, &b);
  if (rc || !e) return rc;
  uint64_t n = 0;
  if (!(rc = rsk_bitset_strlen(b, &n))) rc = rsk_bitset_clear(b); /* a filter keeps its {name}__config */
  if (!rc && deleted_out) *deleted_out = n > 0;
  release(s, e);
  if (!rc) drop_if_empty(s, name);
  return rc;
}

#define SHIM_MAX_BITOP 16

int rsk_shim_bitset_op(int64_t h, const char *name, int32_t op, const char *const *others, int32_t k) {
  ENTER();
  space *s = sp(h);
  if (!s) return fail("space is null");
  drain(s);
  if (op < RSK_BITOP_AND || op > RSK_BITOP_NOT) return fail("bad BITOP operation");
  if (k < 0 || (k > 0 && !others)) return fail("names is null");
  if (op == RSK_BITOP_NOT && k != 0) return redis_err("ERR BITOP NOT must be called with a single source key.");
  if (k + 1 > SHIM_MAX_BITOP) return fail("at most 15 other names per BITOP");
  /* BITOP op name name others... (RedissonBitSet.java:138-145): the
   * destination and the sources; missing sources read as empty strings */
  entry *es[SHIM_MAX_BITOP + 1];
  rsk_bitset *srcs[SHIM_MAX_BITOP];
  rsk_bitset *empty = NULL;
  int m = 0, rc = RSK_OK;
  for (int32_t j = -1; j < k && rc == RSK_OK; ++j) {
    entry *e;
    rsk_bitset *b;
    rc = bits_entry(s, j < 0 ? name : others[j], 0, &e, &b);
    if (rc) break;
    if (e) es[m] = e;
    else {
      if (!empty && (rc = rsk_bitset_create(s->ctx, &empty))) break;
      b = empty;
      es[m] = NULL;
    }
    srcs[m++] = b;
  }
  entry *d = NULL;
  rsk_bitset *db = NULL;
  if (!rc) rc = bits_entry(s, name, 1, &d, &db);
  if (!rc) rc = rsk_bitset_bitop(op, db, srcs, (uint32_t)m);
  if (d) release(s, d);
  for (int j = 0; j < m; ++j)
    if (es[j]) release(s, es[j]);
  if (empty) (void)rsk_bitset_destroy(empty);
  if (!rc) drop_if_empty(s, name);
  return rc;
}
