/*
 * rsketch_shim.h -- the JNI-independent half of the Java binding of librsketch.so.
 *
 * jni/rsketch_jni.c (compiled only where a JDK provides jni.h) turns each
 * native method of org.redisson.gpu.RSketchNative into one call below: it
 * fetches the direct buffers' addresses and capacities (GetDirectBufferAddress /
 * GetDirectBufferCapacity), calls the shim, and on a non-zero status throws
 * rsk_shim_exception_class(rc) with rsk_shim_last_error() as the message.  Keeping
 * every check, conversion and decision here lets tests/c/shim_caller.c drive
 * exactly the code a JVM would run, with plain C buffers standing in for
 * direct buffers.
 *
 * The keyspace.  Redis resolves every object by NAME: two RHyperLogLog or
 * RBloomFilter instances with one name are one key, PFCOUNT of a missing key
 * is 0 and creates nothing, a Bloom filter's size and k live in the hash
 * {name}__config that any instance (or client) re-reads
 * (RedissonBloomFilter.java:206-221), and a getter on a filter nobody
 * initialised throws IllegalStateException("Bloom filter is not initialized!")
 * (:258-287).  The shim keeps that keyspace next to the GPU context: a space
 * = one rsk_ctx + a name -> object registry (reference counted, thread-safe),
 * so the Java objects hold only their name, exactly like the Redis-backed ones.
 *
 * Handles cross the boundary as jlong (int64_t): the space (rsk_shim_space*).
 */
#ifndef RSKETCH_SHIM_H
#define RSKETCH_SHIM_H
#include <stdint.h>

#include "rsketch.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Shim-level status on top of rsk_status: a Bloom call made with a stale
 * (size, k) -- another client re-initialised the filter.  The reference's Lua
 * guard raises RedisException "Bloom filter config has been changed"
 * (RedissonBloomFilter.java:180-186) and the Java object retries after
 * re-reading {name}__config (:108-112, :162-166). */
#define RSK_SHIM_CONFIG_CHANGED 100
/* Shim-level status: an error reply Redis itself would give (a bit offset
 * outside [0, 2^32), BITOP NOT with other keys): RedisException with Redis's
 * message, as CommandDecoder raises for -ERR (CommandDecoder.java:239-243). */
#define RSK_SHIM_REDIS_ERROR 101

/* A java.nio direct buffer as JNI reports it: address + capacity in ELEMENTS
 * (bytes for a ByteBuffer, longs for a LongBuffer).  addr == NULL means the
 * Java side passed a heap (non-direct) buffer or null. */
typedef struct rsk_shim_buf {
  void *addr;
  int64_t cap;
} rsk_shim_buf;

/* The exception the reference raises for a status (see rsketch.h rsk_status):
 * "java/lang/IllegalArgumentException", "java/lang/IllegalStateException",
 * "org/redisson/client/RedisException", "java/lang/OutOfMemoryError";
 * NULL for RSK_OK. */
const char *rsk_shim_exception_class(int rc);
/* The message for the exception: the shim's own when it refused the call,
 * else rsk_last_error() (both thread-local). */
const char *rsk_shim_last_error(void);

/* Key batch from a ByteBuffer of codec-encoded elements back to back and a
 * LongBuffer (native byte order) of n+1 offsets.  Refuses (IllegalArgument)
 * non-direct buffers, n < 0, fewer than n+1 offsets, decreasing offsets, and
 * offsets outside [0, keys.cap]: the library reads raw memory, so a bad Java
 * buffer must stop here, not fault in a kernel. */
int rsk_shim_keys(rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n, rsk_keys *out);

/* ------------------------------------------------------------- space */
/* One GPU context and its keyspace.  extended_bloom: tryInit sizes above
 * RedissonBloomFilter.MAX_SIZE are allowed (RSK_BLOOM_EXTENDED) instead of
 * refused with IllegalArgumentException like the reference (:226-227). */
int rsk_shim_init(int32_t device, int32_t extended_bloom, int64_t *space_out);
int rsk_shim_shutdown(int64_t space);
/* The library context of a space (for callers of the C ABI itself, e.g. the
 * support library of include/rsketch_diag.h); NULL for a null space. */
rsk_ctx *rsk_shim_context(int64_t space);
/* Waits until every call issued so far has completed and its callback has
 * returned (rsk_sync).  Callbacks may call the shim again (rsketch.h,
 * rsk_done_fn): this wait does not hold the context. */
int rsk_shim_sync(int64_t space);

#define RSK_SHIM_NONE 0
#define RSK_SHIM_HLL 1
#define RSK_SHIM_BLOOM 2
#define RSK_SHIM_BITSET 3
/* TYPE-like probe of a name (RSK_SHIM_NONE / _HLL / _BLOOM / _BITSET) and the object's
 * library handle (the same handle for every lookup of one name; 0 if none). */
int rsk_shim_lookup(int64_t space, const char *name, int32_t *type_out, int64_t *handle_out);
/* DEL name (a Bloom filter's {name}__config with it, RedissonBloomFilter.java:
 * 201-204); *deleted_out = 1 iff something existed.  Calls still running on
 * the object finish first; the object is released after the last of them. */
int rsk_shim_delete(int64_t space, const char *name, int32_t *deleted_out);

/* RENAME / RENAMENX old new (RedissonObject.java:72-110): the object moves to
 * the new name (a Bloom filter with its config); RENAME replaces an object
 * the new name held, RENAMENX leaves both and answers 0 then.  A missing old
 * name is RSK_ERR_INVALID_ARG ("ERR no such key"). *renamed_out may be NULL. */
int rsk_shim_rename(int64_t space, const char *old_name, const char *new_name, int32_t nx, int32_t *renamed_out);

/* --------------------------------- RHyperLogLog (RedissonHyperLogLog.java:40-97) */
/* PFADD name e1..en (creates the key); *changed_out = the reply. */
int rsk_shim_hll_add(int64_t space, const char *name, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                     uint8_t *changed_out);
/* n x PFADD name e (RBatch of add()s); replies: n bytes (jboolean == uint8_t). */
int rsk_shim_hll_add_each(int64_t space, const char *name, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                          uint8_t *replies, int64_t replies_len);
/* PFCOUNT name: 0 for a missing key, which stays missing. */
int rsk_shim_hll_count(int64_t space, const char *name, int64_t *out);
/* PFCOUNT names[0..k): missing keys are skipped (all missing: 0). */
int rsk_shim_hll_count_with(int64_t space, const char *const *names, int32_t k, int64_t *out);
/* PFMERGE dst srcs[0..k): dst created (dense), missing sources skipped. */
int rsk_shim_hll_merge_with(int64_t space, const char *dst, const char *const *srcs, int32_t k);
/* The RBatch of the reference (RedissonBatch.java:76-83 getHyperLogLog, :226-233
 * execute) for add(): element i is "PFADD names[name_of[i]] e_i"; the replies
 * come back in input order.  One rsk_hll_add_each per distinct name, its
 * elements in input order (different keys are independent). */
int rsk_shim_batch_hll_add(int64_t space, const char *const *names, int32_t n_names, const int32_t *name_of,
                           rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n, uint8_t *replies, int64_t replies_len);

/* Asynchronous twins (RHyperLogLogAsync.java:22-33): cb(user, status, value)
 * fires once per accepted call, from the context's completion thread (value: the reply, as
 * rsketch.h's rsk_done_fn); a refused call returns the error and never fires.
 * A count of a missing key fires on the calling thread with 0. */
int rsk_shim_hll_add_async(int64_t space, const char *name, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                           rsk_done_fn cb, void *user);
int rsk_shim_hll_count_async(int64_t space, const char *name, rsk_done_fn cb, void *user);
int rsk_shim_hll_count_with_async(int64_t space, const char *const *names, int32_t k, rsk_done_fn cb, void *user);
int rsk_shim_hll_merge_with_async(int64_t space, const char *dst, const char *const *srcs, int32_t k, rsk_done_fn cb,
                                  void *user);

/* ------------------------------ RBloomFilter (RedissonBloomFilter.java:52-287) */
/* The {name}__config hash (:237-240). */
typedef struct rsk_shim_bloom_config {
  int64_t size;
  int32_t hash_iterations;
  int64_t expected_insertions;
  double false_probability;
} rsk_shim_bloom_config;
/* tryInit(n, p) (:223-252): the size is computed first (IllegalArgument above
 * MAX_SIZE in compat mode, as the reference throws before looking at Redis);
 * then *created_out = 1 and a zeroed filter if the name has no config, else 0
 * and the stored config (the reference's readConfig on "config has been
 * changed").  cfg_out (may be NULL) = the config in force after the call. */
int rsk_shim_bloom_try_init(int64_t space, const char *name, int64_t expected_insertions, double false_probability,
                            int32_t *created_out, rsk_shim_bloom_config *cfg_out);
/* HGETALL {name}__config: RSK_ERR_NOT_INITIALIZED when absent (getSize,
 * getHashIterations, getExpectedInsertions, getFalseProbability, :258-287). */
int rsk_shim_bloom_get_config(int64_t space, const char *name, rsk_shim_bloom_config *out);
/* add / contains / count with the caller's cached (size, k), like the
 * reference's batch with its Lua config guard: a missing filter is
 * RSK_ERR_NOT_INITIALIZED (:206-221), a different stored config
 * RSK_SHIM_CONFIG_CHANGED (re-read, retry).  add's replies: 1 iff one of the
 * first k-1 SETBITs found its bit clear (:100-107); contains: AND of the
 * first k-1 GETBITs (:147-168); replies / out NULL allowed for add only. */
int rsk_shim_bloom_add(int64_t space, const char *name, int64_t size, int32_t k, rsk_shim_buf keys,
                       rsk_shim_buf offsets, int64_t n, uint8_t *replies, int64_t replies_len);
int rsk_shim_bloom_contains(int64_t space, const char *name, int64_t size, int32_t k, rsk_shim_buf keys,
                            rsk_shim_buf offsets, int64_t n, uint8_t *out, int64_t out_len);
/* count() (:188-199): config and BITCOUNT read together. */
int rsk_shim_bloom_count(int64_t space, const char *name, int32_t *out);
int rsk_shim_bloom_add_async(int64_t space, const char *name, int64_t size, int32_t k, rsk_shim_buf keys,
                             rsk_shim_buf offsets, int64_t n, uint8_t *replies, int64_t replies_len, rsk_done_fn cb,
                             void *user);
int rsk_shim_bloom_contains_async(int64_t space, const char *name, int64_t size, int32_t k, rsk_shim_buf keys,
                                  rsk_shim_buf offsets, int64_t n, uint8_t *out, int64_t out_len, rsk_done_fn cb,
                                  void *user);

/* ------------------------------------ RBitSet (RedissonBitSet.java:32-270) */
/* getBitSet(name) (Redisson.java:515-517; RBatch.getBitSet, RedissonBatch.java:
 * 191) on the keyspace.  The name holds a plain string (made by the first
 * write), or a Bloom filter -- whose bits ARE the string key in Redis, so
 * these calls read and write the filter's bits (rsk_bloom_bitset: GET returns
 * exactly the bytes Redis would) -- or nothing (an empty string: GET nil,
 * GETBIT / BITCOUNT / length 0).  An HLL name is WRONGTYPE.  Offsets outside
 * [0, 2^32) are RSK_SHIM_REDIS_ERROR, as Redis replies. */
int rsk_shim_bitset_strlen(int64_t space, const char *name, int64_t *bytes_out); /* size() = 8 * STRLEN */
/* GET (toByteArray, :88-91): *bytes_out malloc'd (free with rsk_shim_free),
 * *len_out = -1 and NULL for a missing key (nil). */
int rsk_shim_bitset_get_bytes(int64_t space, const char *name, uint8_t **bytes_out, int64_t *len_out);
void rsk_shim_free(void *p);
int rsk_shim_bitset_getbits(int64_t space, const char *name, const int64_t *offsets, int64_t n, uint8_t *out,
                            int64_t out_len);                                          /* GETBIT x n */
int rsk_shim_bitset_setbits(int64_t space, const char *name, const int64_t *offsets, int64_t n, int32_t value);
int rsk_shim_bitset_set_range(int64_t space, const char *name, int64_t from, int64_t to, int32_t value);
int rsk_shim_bitset_cardinality(int64_t space, const char *name, int64_t *out);       /* BITCOUNT */
int rsk_shim_bitset_length(int64_t space, const char *name, int64_t *out);            /* length() */
int rsk_shim_bitset_set_bytes(int64_t space, const char *name, const uint8_t *bytes, int64_t len); /* SET */
/* clear() = DEL name: a plain string goes away; a Bloom filter's bits are
 * zeroed and its {name}__config stays (DEL removes only the string key).
 * *deleted_out (may be NULL) = 1 iff a non-empty string existed. */
int rsk_shim_bitset_clear(int64_t space, const char *name, int32_t *deleted_out);
/* BITOP op name name others[0..k) (or/and/xor/not, :125-145,216-268; op as
 * rsk_bitop, NOT with k = 0). */
int rsk_shim_bitset_op(int64_t space, const char *name, int32_t op, const char *const *others, int32_t k);

#ifdef __cplusplus
}
#endif
#endif /* RSKETCH_SHIM_H */
