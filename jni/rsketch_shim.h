/*
 * rsketch_shim.h -- the JNI-independent half of the Java binding of librsketch.so.
 *
 * jni/rsketch_jni.c (compiled only where a JDK provides jni.h) turns each
 * native method of org.redisson.gpu.RSketchNative into one call below: it
 * fetches the direct buffers' addresses and capacities (GetDirectBufferAddress /
 * GetDirectBufferCapacity), calls the shim, and on a non-zero status throws
 * rsk_shim_exception_class(rc) with rsk_last_error() as the message.  Keeping
 * every check and conversion here lets tests/c/shim_caller.c drive exactly the
 * code a JVM would run, with plain C buffers standing in for direct buffers.
 *
 * Handles cross the boundary as jlong (int64_t): rsk_ctx* / rsk_hll* / rsk_bloom*.
 */
#ifndef RSKETCH_SHIM_H
#define RSKETCH_SHIM_H
#include <stdint.h>

#include "rsketch.h"

#ifdef __cplusplus
extern "C" {
#endif

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

int rsk_shim_init(int32_t device, int64_t *ctx_out);
int rsk_shim_shutdown(int64_t ctx);

/* RHyperLogLog (RedissonHyperLogLog.java:40-97) */
int rsk_shim_hll_create(int64_t ctx, int64_t n_sketches, int64_t *hll_out);
int rsk_shim_hll_destroy(int64_t hll);
int rsk_shim_hll_add(int64_t hll, int64_t id, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                     uint8_t *changed_out);
/* replies: n bytes (the jbooleanArray region, jboolean == uint8_t) */
int rsk_shim_hll_add_each(int64_t hll, int64_t id, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n,
                          uint8_t *replies, int64_t replies_len);
int rsk_shim_hll_count(int64_t hll, int64_t id, int64_t *out);
/* countWith: k >= 1 (pool, id) members; mergeWith: dst <- max(dst, srcs) */
int rsk_shim_hll_count_union(const int64_t *hlls, const int64_t *ids, int32_t k, int64_t *out);
int rsk_shim_hll_merge(int64_t dst, int64_t dst_id, const int64_t *srcs, const int64_t *src_ids, int32_t k);
int rsk_shim_hll_delete(int64_t hll, int64_t id);

/* RBloomFilter (RedissonBloomFilter.java:52-252) */
int rsk_shim_bloom_params(int64_t expected_insertions, double false_probability, int32_t extended,
                          int64_t *size_out, int32_t *k_out);
int rsk_shim_bloom_create(int64_t ctx, int64_t size, int32_t k, int64_t *bloom_out);
int rsk_shim_bloom_destroy(int64_t bloom);
int rsk_shim_bloom_add(int64_t bloom, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n, uint8_t *replies,
                       int64_t replies_len);
int rsk_shim_bloom_contains(int64_t bloom, rsk_shim_buf keys, rsk_shim_buf offsets, int64_t n, uint8_t *out,
                            int64_t out_len);
int rsk_shim_bloom_count(int64_t bloom, int32_t *out);

#ifdef __cplusplus
}
#endif
#endif /* RSKETCH_SHIM_H */
