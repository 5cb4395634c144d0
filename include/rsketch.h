/*
 * rsketch.h -- C ABI of librsketch.so, the MI355X (gfx950) sketch engine
 * behind Redisson's RHyperLogLog / RBloomFilter / RBitSet.
 *
 * The reference (alexs20/redisson, Redisson 2.2.17) has no native layer: its
 * operator interface for this path is the Java object API, which today sends
 * PFADD/PFCOUNT/PFMERGE/SETBIT/GETBIT/BITCOUNT to a Redis server.  Each entry
 * point below replaces one of those Java methods (cited file:line, paths
 * relative to src/main/java/org/redisson/) and is what a JNI shim binds
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every function returns an rsk_status; details via rsk_last_error()
 *    (thread-local).  Status codes map 1:1 to the Java exceptions the
 *    reference raises (see enum).  No C++ exception crosses this boundary.
 *  - The caller owns all buffers passed in.  Key buffers live either in host
 *    memory (RSK_MEM_HOST; copied over PCIe through two pinned host stages,
 *    filled by host threads -- rsk_options.stage_threads, default 8 -- while
 *    the other stage's DMA runs) or in device memory of the context's GPU
 *    (RSK_MEM_DEVICE; read in place).  Per-key outputs follow the keys'
 *    location; a RSK_MEM_DEVICE key or output pointer the GPU cannot reach
 *    (pageable host memory) is refused with RSK_ERR_INVALID_ARG.
 *  - The library owns device state behind opaque handles.  Calls on one
 *    context are serialised on that context's HIP stream; results written to
 *    host pointers are complete when the call returns.
 *  - HLL semantics are Redis 3.2.0's (the version the reference CI pins,
 *    .travis.yml:24): 16384 six-bit registers, MurmurHash64A seed
 *    0xadc83b19, rank in [1,50], the 3.2.0 estimator.
 */
#ifndef RSKETCH_H
#define RSKETCH_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* librsketch.so is built with hidden visibility: exactly the functions
 * declared here are exported. */
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

/* rsk_abi_version() returns this; a caller built against another header must
 * not call in.  2: rsk_options is 24 bytes (stage_threads, reserved) and the
 * asynchronous entry points exist (1 had a 16-byte rsk_options). */
#define RSK_ABI_VERSION 2
#define RSK_HLL_REGISTERS 16384
#define RSK_HLL_DENSE_BYTES 12304 /* 16-byte "HYLL" header + 12288 register bytes */

typedef enum rsk_status {
  RSK_OK = 0,
  RSK_ERR_INVALID_ARG = 1,     /* IllegalArgumentException (RedissonBloomFilter.java:175,227) */
  RSK_ERR_NOT_INITIALIZED = 2, /* IllegalStateException "Bloom filter is not initialized!" (:217,:284) */
  RSK_ERR_WRONGTYPE = 3,       /* RedisException -WRONGTYPE (CommandDecoder.java:239-243) */
  RSK_ERR_INVALID_HLL = 4,     /* RedisException -INVALIDOBJ Corrupted HLL object */
  RSK_ERR_DEVICE = 5,          /* HIP runtime / kernel failure */
  RSK_ERR_OUT_OF_MEMORY = 6,   /* device allocation failed */
  RSK_ERR_NO_DEVICE = 7        /* no gfx950 device visible */
} rsk_status;

typedef enum rsk_mem { RSK_MEM_HOST = 0, RSK_MEM_DEVICE = 1 } rsk_mem;

typedef struct rsk_ctx rsk_ctx;
typedef struct rsk_hll rsk_hll;
typedef struct rsk_bloom rsk_bloom;

typedef struct rsk_options {
  int32_t device;         /* HIP device ordinal (one process per GPU) */
  int32_t redis_version;  /* 320 = Redis 3.2.0 semantics (only supported value) */
  uint64_t staging_bytes; /* bytes per host->device chunk (each of the two pinned
                             stages holds one chunk + its offsets); 0 = default (256 MiB) */
  uint32_t stage_threads; /* host threads filling a pinned stage; 0 = default (8) */
  uint32_t reserved;      /* must be 0 */
} rsk_options;

/* A batch of keys: fixed stride (offsets == NULL, each key fixed_len bytes)
 * or a blob with n+1 byte offsets (key i = data[offsets[i] .. offsets[i+1])).
 * data and offsets share one location.  These are the codec-encoded element
 * bytes (CommandEncoder.java:77-79 / RedissonBloomFilter.java:170-178). */
typedef struct rsk_keys {
  const void *data;
  const uint64_t *offsets;
  uint64_t n;
  uint32_t fixed_len;
  uint32_t location; /* rsk_mem */
} rsk_keys;

/* Completion callback of the asynchronous entry points (rsk_*_async), the
 * C side of RHyperLogLogAsync / RBloomFilter futures (RHyperLogLogAsync.java:
 * 22-33; CommandAsyncService.java:86-105 completes a Netty promise the same
 * way).  status: RSK_OK (the call's device work finished) or RSK_ERR_DEVICE
 * (a device error on the context's streams: value 0, per-key outputs not
 * written, and every later call on the context fails with RSK_ERR_DEVICE);
 * value: the reply -- PFADD's changed flag (0/1), PFCOUNT's count, the number
 * of keys of a Bloom add/contains whose per-key outputs are in place.  It runs
 * once per accepted call on the context's completion thread, in submission
 * order (the stream only queues it there, so a slow callback does not hold up
 * later device work).  A callback may call librsketch again, synchronously or
 * asynchronously, on any context -- except rsk_shutdown of its own context; a
 * call it makes runs while later callbacks wait, so a callback that blocks on
 * the completion of a LATER asynchronous call of its own context deadlocks
 * (as a Netty listener that blocks on its own event loop does).  rsk_sync
 * returns after the callbacks of every call issued before it have returned
 * (it does not hold the context while it waits for them). */
typedef void (*rsk_done_fn)(void *user, int status, uint64_t value);

/* ---------------------------------------------------------------- context */
int rsk_init(const rsk_options *opts, rsk_ctx **out);
int rsk_shutdown(rsk_ctx *ctx);
const char *rsk_last_error(void);
int rsk_abi_version(void);
/* The HIP stream (hipStream_t) every call on this context is ordered on. */
void *rsk_ctx_stream(rsk_ctx *ctx);
int rsk_sync(rsk_ctx *ctx);
/* Release the context's grow-on-demand scratch (device work and output
 * buffers, pinned per-op buffer).  Large batches grow it (the add()-with-
 * replies pipeline up to ~165 GB at 1B keys); it is kept for the next call
 * otherwise.  Waits for the context's queued work. */
int rsk_trim(rsk_ctx *ctx);
/* Pin a caller's pageable host buffer in place (hipHostRegister) for as long
 * as the caller keeps it registered -- a long-lived buffer reused across calls,
 * like a Java direct ByteBuffer holding checkpoints.  The batched export /
 * import (rsk_hll_export_redis_batch / import_redis_batch) and staged key
 * batches then move data between HBM and a registered range by DMA straight
 * to / from it, instead of through the library's pinned stages and a host
 * copy.  A range may not overlap one already registered; rsk_host_unregister
 * takes the pointer given to rsk_host_register; rsk_shutdown unregisters what
 * is left. */
int rsk_host_register(rsk_ctx *ctx, void *ptr, uint64_t bytes);
int rsk_host_unregister(rsk_ctx *ctx, void *ptr);
/* Per-kernel device-time accounting with HIP events on the context stream
 * (used by bench.py for the roofline; off by default). */
int rsk_prof_enable(rsk_ctx *ctx, int on);
int rsk_prof_reset(rsk_ctx *ctx);
/* Accumulated milliseconds and launch count of kernel `name` since reset. */
int rsk_prof_read(rsk_ctx *ctx, const char *name, double *ms, uint64_t *launches);

/* ------------------------------------------------------------ HyperLogLog */
/* A pool of n_sketches HLL keys (n_sketches = 1 for RHyperLogLog; 1e6 for
 * the grouped COUNT DISTINCT config).  Sketches start absent (no key). */
int rsk_hll_create(rsk_ctx *ctx, uint64_t n_sketches, rsk_hll **out);
int rsk_hll_destroy(rsk_hll *h);
uint64_t rsk_hll_size(const rsk_hll *h);
/* 1 if the sketch exists (was created by add/merge/import), else 0. */
int rsk_hll_exists(rsk_hll *h, uint64_t id, int *out);
/* DEL: RedissonObject.deleteAsync (RedissonObject.java:117-119). */
int rsk_hll_delete(rsk_hll *h, uint64_t id);
/* DEL of every sketch in the pool (registers and caches zeroed). */
int rsk_hll_clear(rsk_hll *h);

/* PFADD id e1..en -- RedissonHyperLogLog.addAll/addAllAsync (:46-48,:70-76)
 * with the INTENDED semantics (the fork's varargs bug is not reproduced, see
 * DESIGN.md).  *changed_out (may be NULL) = 1 iff any register grew or the
 * key was created: BooleanReplayConvertor (BooleanReplayConvertor.java:20-26). */
int rsk_hll_add(rsk_hll *h, uint64_t id, const rsk_keys *keys, uint8_t *changed_out);

/* One PFADD per element, in input order -- RedissonHyperLogLog.add (:40-43)
 * issued n times (e.g. pipelined in an RBatch, RedissonBatch.java:76-83).
 * out[i] = the reply of the i-th PFADD. */
int rsk_hll_add_each(rsk_hll *h, uint64_t id, const rsk_keys *keys, uint8_t *out);

/* Grouped PFADD: element i goes to sketch groups[i] (group ids in the same
 * location as the keys).  Grouped COUNT DISTINCT (BASELINE config 5). */
int rsk_hll_add_grouped(rsk_hll *h, const rsk_keys *keys, const uint32_t *groups);

/* PFCOUNT id -- RedissonHyperLogLog.count/countAsync (:50-53,:78-81), for
 * n ids at once; out is a host array of n uint64.  Honours and refreshes the
 * per-key cardinality cache exactly like pfcountCommand. */
int rsk_hll_count(rsk_hll *h, const uint64_t *ids, uint64_t n, uint64_t *out);

/* PFCOUNT k1..kk (k >= 2 keys may repeat, pools may differ) --
 * RedissonHyperLogLog.countWith/countWithAsync (:55-58,:83-89). */
int rsk_hll_count_union(rsk_hll *const *hs, const uint64_t *ids, uint32_t k, uint64_t *out);
/* Batched countWith: n unions of `arity` members each, all in pool h;
 * member_ids is [n][arity] (host); out is [n]. */
int rsk_hll_count_union_batch(rsk_hll *h, const uint64_t *member_ids, uint32_t arity, uint64_t n,
                              uint64_t *out);

/* PFMERGE dst src1..srck (dst included in the max) --
 * RedissonHyperLogLog.mergeWith/mergeWithAsync (:60-63,:91-97). */
int rsk_hll_merge(rsk_hll *dst, uint64_t dst_id, rsk_hll *const *srcs, const uint64_t *src_ids, uint32_t k);
/* Batched mergeWith within one pool: for i < n, PFMERGE dst_ids[i] src_ids[i],
 * in input order.  Returns when the merges are done (rsk_hll_merge_batch_async
 * returns once they are queued). */
int rsk_hll_merge_batch(rsk_hll *h, const uint64_t *dst_ids, const uint64_t *src_ids, uint64_t n);

/* Asynchronous twins (RHyperLogLogAsync: addAllAsync, countAsync,
 * countWithAsync, mergeWithAsync; RedissonHyperLogLog.java:65-97).  Arguments
 * are validated and the work enqueued on the context stream before the call
 * returns (RSK_OK: cb fires exactly once later; any other status: it never
 * fires).  Host key batches are copied into the call's own pinned buffer, so
 * the caller may reuse them at once; batches above 256 MiB run before the
 * call returns and cb fires on the calling thread.  Calls on different
 * handles may be issued from any threads concurrently; every call is ordered
 * on its context's stream like the synchronous ones. */
int rsk_hll_add_async(rsk_hll *h, uint64_t id, const rsk_keys *keys, rsk_done_fn cb, void *user);
int rsk_hll_count_async(rsk_hll *h, uint64_t id, rsk_done_fn cb, void *user);
int rsk_hll_count_union_async(rsk_hll *const *hs, const uint64_t *ids, uint32_t k, rsk_done_fn cb, void *user);
int rsk_hll_merge_async(rsk_hll *dst, uint64_t dst_id, rsk_hll *const *srcs, const uint64_t *src_ids, uint32_t k,
                        rsk_done_fn cb, void *user);
int rsk_hll_merge_batch_async(rsk_hll *h, const uint64_t *dst_ids, const uint64_t *src_ids, uint64_t n,
                              rsk_done_fn cb, void *user);
/* Pool forms (a pipelined batch of the grouped calls above): grouped PFADD
 * (value n), PFCOUNT of ids (NULL: sketches 0..n-1) and batched countWith
 * into out (value n).  out is written before cb fires; keep it alive until
 * then.  Members of a countWith are taken as they stand at that point of the
 * call order, exactly like the synchronous call issued there. */
int rsk_hll_add_grouped_async(rsk_hll *h, const rsk_keys *keys, const uint32_t *groups, rsk_done_fn cb, void *user);
int rsk_hll_count_ids_async(rsk_hll *h, const uint64_t *ids, uint64_t n, uint64_t *out, rsk_done_fn cb, void *user);
int rsk_hll_count_union_batch_async(rsk_hll *h, const uint64_t *member_ids, uint32_t arity, uint64_t n,
                                    uint64_t *out, rsk_done_fn cb, void *user);

/* PFMERGE from raw registers (one byte per register, any location): the
 * receive side of the multi-GPU RCCL MAX merge. */
int rsk_hll_merge_raw(rsk_hll *h, uint64_t id, const uint8_t *regs, uint32_t location);
/* Raw registers out (host or device destination, 16384 bytes). */
int rsk_hll_get_registers(rsk_hll *h, uint64_t id, uint8_t *out, uint32_t location);
/* Device pointer of the [n_sketches][16384] register array (for RCCL).  A
 * caller that writes registers through it must do so before its next call on
 * this pool (each call re-derives the pool's cached state from that point). */
void *rsk_hll_device_registers(rsk_hll *h);

/* GET of the key as a Redis "HYLL" string, in the encoding Redis 3.2 would
 * hold it in: SPARSE (16-byte header + canonical opcodes, at most
 * hll-sparse-max-bytes = 3000 bytes) while the key never left the sparse
 * encoding, else DENSE (12304 bytes; dense for good once promoted, after
 * PFMERGE and after a multi-GPU merge); a string SET by rsk_hll_import_redis
 * and not written since comes back byte for byte.  Card bytes as Redis would
 * hold them.  cap must be >= 12304; *len = 0 for a missing key (nil).
 * RBitSet.toByteArray-style export. */
int rsk_hll_export_redis(rsk_hll *h, uint64_t id, uint8_t *buf, size_t cap, size_t *len);
/* SET of a Redis HLL string (dense or sparse); validated like
 * isHLLObjectOrReply / hllMerge.  Replaces the key. */
int rsk_hll_import_redis(rsk_hll *h, uint64_t id, const uint8_t *buf, size_t len);

/* Batched GET: for each ids[i] the bytes rsk_hll_export_redis returns (empty
 * for a missing key), packed back to back into out (host memory, cap bytes);
 * key i occupies out[offsets[i] .. offsets[i+1]) (offsets: n + 1 entries).
 * Same encoding decisions as the per-key call (sparse while the key fits,
 * promoted for good otherwise; kept SET strings byte for byte); the sparse
 * opcodes and the 6-bit dense packing are produced on the device, one wave
 * per key, each key encoded once, one copy per 65536 keys -- the checkpoint
 * of a pool.  cap too small: RSK_ERR_INVALID_ARG with offsets
 * filled (offsets[n] = the bytes needed); out holds at most the strings of
 * the whole chunks of 65536 keys that fit before the first that does not. */
int rsk_hll_export_redis_batch(rsk_hll *h, const uint64_t *ids, uint64_t n, uint8_t *out, uint64_t cap,
                               uint64_t *offsets);
/* Batched SET: key ids[i] := the Redis HLL string data[offsets[i] .. offsets[i+1])
 * (host memory; offsets: n + 1 non-decreasing entries), each validated like
 * rsk_hll_import_redis.  All or nothing: one invalid string fails the call
 * (RSK_ERR_WRONGTYPE / RSK_ERR_INVALID_HLL, its index in the message) before
 * any key changes.  A key SET twice in one call keeps the later string. */
int rsk_hll_import_redis_batch(rsk_hll *h, const uint64_t *ids, uint64_t n, const uint8_t *data,
                               const uint64_t *offsets);

/* ---------------------------------------------------------- Bloom filter */
typedef enum rsk_bloom_mode {
  RSK_BLOOM_COMPAT = 0,  /* size <= 2*Integer.MAX_VALUE (RedissonBloomFilter.java:52,226-227) */
  RSK_BLOOM_EXTENDED = 1 /* larger filters (1B @ 1% = 9,585,058,377 bits) */
} rsk_bloom_mode;

/* tryInit sizing (optimalNumOfBits / optimalNumOfHashFunctions,
 * RedissonBloomFilter.java:69-78,223-229) without allocating. */
int rsk_bloom_params(int64_t expected_insertions, double false_probability, uint32_t mode,
                     int64_t *size_out, int32_t *k_out);
/* Allocate a zeroed filter of explicit size/k (the {name}__config values). */
int rsk_bloom_create(rsk_ctx *ctx, int64_t size, int32_t k, rsk_bloom **out);
/* tryInit(n, p): params + create. */
int rsk_bloom_init(rsk_ctx *ctx, int64_t expected_insertions, double false_probability, uint32_t mode,
                   rsk_bloom **out, int64_t *size_out, int32_t *k_out);
int rsk_bloom_destroy(rsk_bloom *b);
int rsk_bloom_info(const rsk_bloom *b, int64_t *size, int32_t *k);
/* add(obj) for n objects in input order (RedissonBloomFilter.java:80-114).
 * added_out (may be NULL; host memory for RSK_MEM_HOST batches, device memory
 * for RSK_MEM_DEVICE ones) gets each add's reply: 1 iff one of the first k-1
 * SETBITs found its bit clear, exactly as if the adds ran one by one in input
 * order.  Large batches answer through the first-key partition pipeline
 * (DESIGN.md section 3), small ones through a sort of (bit, sequence). */
int rsk_bloom_add(rsk_bloom *b, const rsk_keys *keys, uint8_t *added_out);
/* contains(obj) for n objects (RedissonBloomFilter.java:133-168): 1 iff the
 * first k-1 bits are all set.  out is a host array of n bytes. */
int rsk_bloom_contains(rsk_bloom *b, const rsk_keys *keys, uint8_t *out);
/* count() (RedissonBloomFilter.java:188-199) and the BITCOUNT it uses. */
int rsk_bloom_count(rsk_bloom *b, int32_t *out);
int rsk_bloom_bitcount(rsk_bloom *b, uint64_t *out);

/* Asynchronous add / contains (the futures of RBloomFilter's batch calls):
 * conventions as for rsk_hll_add_async; per-key outputs are in place when cb
 * fires (host outputs must stay valid until then). */
int rsk_bloom_add_async(rsk_bloom *b, const rsk_keys *keys, uint8_t *added_out, rsk_done_fn cb, void *user);
int rsk_bloom_contains_async(rsk_bloom *b, const rsk_keys *keys, uint8_t *out, rsk_done_fn cb, void *user);

/* Hash.hashToBase64 (src/main/java/org/redisson/misc/Hash.java:29-40) of each
 * key: farmUo and xx_r39 as two big-endian longs, Base64, trailing "=="
 * dropped -> 22 ASCII chars per key, key i at out + 22*i (no terminators).
 * `out` is in the keys' location. */
int rsk_hash_to_base64(rsk_ctx *ctx, const rsk_keys *keys, char *out);
/* The bit string as Redis holds it (MSB-first, ceil(size/8) bytes). */
int rsk_bloom_export_bits(rsk_bloom *b, uint8_t *buf, size_t cap, size_t *len);
int rsk_bloom_import_bits(rsk_bloom *b, const uint8_t *buf, size_t len);
/* OR raw bitset bytes (any location, ceil(size/8) bytes) into the filter:
 * the receive side of the multi-GPU slice-OR merge. */
int rsk_bloom_or_bits(rsk_bloom *b, const uint8_t *bits, size_t len, uint32_t location);
void *rsk_bloom_device_bits(rsk_bloom *b);

/* --------------------------------------------------------------- RBitSet */
/* A Redis string addressed as bits, MSB-first (bitops.c; the layout the
 * Bloom filter uses).  Each call replaces the command RedissonBitSet sends
 * (src/main/java/org/redisson/RedissonBitSet.java). */
typedef struct rsk_bitset rsk_bitset;
typedef enum rsk_bitop { RSK_BITOP_AND = 0, RSK_BITOP_OR = 1, RSK_BITOP_XOR = 2, RSK_BITOP_NOT = 3 } rsk_bitop;
int rsk_bitset_create(rsk_ctx *ctx, rsk_bitset **out);  /* an absent key (empty string) */
int rsk_bitset_destroy(rsk_bitset *b);
/* STRLEN: size() = 8 * STRLEN (BitsSizeReplayConvertor.java:21-27). */
int rsk_bitset_strlen(rsk_bitset *b, uint64_t *bytes);
/* SETBIT off value for n offsets (set/clear(index) :70-80,:196-209); grows the
 * string to (max offset >> 3) + 1 bytes like Redis.  offsets host or device. */
int rsk_bitset_setbits(rsk_bitset *b, const uint64_t *offsets, uint64_t n, int value, uint32_t location);
/* GETBIT for n offsets (get(index)); out in the offsets' location. */
int rsk_bitset_getbits(rsk_bitset *b, const uint64_t *offsets, uint64_t n, uint32_t location, uint8_t *out);
/* set(from, to) / clear(from, to) (:217-236): SETBIT i v for i in [from, to). */
int rsk_bitset_set_range(rsk_bitset *b, uint64_t from, uint64_t to, int value);
/* BITCOUNT (cardinality(), :240-243). */
int rsk_bitset_bitcount(rsk_bitset *b, uint64_t *out);
/* length(): index of the highest set bit + 1 (0 when none). */
int rsk_bitset_length(rsk_bitset *b, uint64_t *out);
/* BITOP op dst src1..srck (and/or/xor(names) apply it as BITOP op self self
 * names, :125-145; not() as BITOP NOT self self).  dst may be a source. */
int rsk_bitset_bitop(int op, rsk_bitset *dst, rsk_bitset *const *srcs, uint32_t k);
/* GET (toByteArray(), :88-91) / SET (set(BitSet), :211-214) / DEL (clear()). */
int rsk_bitset_get_bytes(rsk_bitset *b, uint8_t *buf, size_t cap, size_t *len);
int rsk_bitset_set_bytes(rsk_bitset *b, const uint8_t *buf, size_t len);
int rsk_bitset_clear(rsk_bitset *b);
/* A Bloom filter's bit string as an RBitSet.  In Redis the filter's bits ARE
 * the string key `name` (RedissonBloomFilter SETBITs it, RedissonBitSet GETs
 * it), so getBitSet(filterName) -- Redisson.java:515-517, RedissonBatch.java:191
 * -- reads and writes them: every rsk_bitset_* call above works on the view.
 * STRLEN is Redis's (the highest byte a SETBIT touched + 1: for the filter's
 * own adds, which only set bits, the last non-zero byte + 1), so GET returns
 * the bytes Redis would; writes through the view change the filter.  The view
 * cannot grow the string past the filter's ceil(size/8) bytes (such a SETBIT /
 * SET / BITOP is refused with RSK_ERR_INVALID_ARG).  rsk_bitset_destroy of
 * the view releases only the view; destroy every view before its filter. */
int rsk_bloom_bitset(rsk_bloom *b, rsk_bitset **out);

/* ------------------------------------------------------- device memory */
/* HBM buffers for keys / replies that stay resident (JNI: wrap as direct
 * buffers; Python: redisson_amd.devmem.DeviceBuffer). */
typedef enum rsk_copy { RSK_H2D = 0, RSK_D2H = 1, RSK_D2D = 2 } rsk_copy;
int rsk_dev_alloc(rsk_ctx *ctx, uint64_t bytes, void **out);
int rsk_dev_free(rsk_ctx *ctx, void *p);
/* Ordered on the context stream; returns when the copy is complete. */
int rsk_memcpy(rsk_ctx *ctx, void *dst, const void *src, uint64_t bytes, uint32_t kind);
int rsk_memset(rsk_ctx *ctx, void *p, int value, uint64_t bytes);

/* ------------------------------------------- multi-GPU (RCCL over xGMI) */
/* One process per GPU.  Rank 0 creates the id, the caller ships it to the
 * other ranks (any out-of-band channel: torch.distributed gloo, MPI, a
 * socket), every rank calls rsk_comm_init.  The key stream is sharded
 * across ranks; the only exchange step is the sketch merge below. */
#define RSK_COMM_ID_BYTES 128
int rsk_comm_unique_id(uint8_t *id_out);
int rsk_comm_init(rsk_ctx *ctx, int nranks, int rank, const uint8_t *id);
int rsk_comm_destroy(rsk_ctx *ctx);
/* The communicator as RCCL reports it (ncclCommCount / ncclCommUserRank), so
 * a caller can check that every rank joined; 1 and 0 without one. */
int rsk_comm_info(rsk_ctx *ctx, int *nranks, int *rank);
/* Sketch id := register-wise MAX over all ranks (ncclAllReduce uint8 MAX,
 * in place, 16 KiB).  Equals PFMERGE of the ranks' sketches; the cache is
 * invalidated. */
int rsk_hll_allreduce(rsk_hll *h, uint64_t id);
/* The whole pool ([n][16384]) MAX over ranks. */
int rsk_hll_allreduce_pool(rsk_hll *h);
/* Grouped pools (C5): ncclReduceScatter(uint8 MAX) in place.  Afterwards this
 * rank's sketches [*first, *first + *count) hold the MAX over all ranks;
 * rank r owns [r*q, (r+1)*q) with q = n / nranks, and the last rank also the
 * n mod nranks tail (which is all-reduced on every rank).  Sketches outside
 * the owned range keep this rank's partial registers.  Caches invalidated. */
int rsk_hll_reducescatter_pool(rsk_hll *h, uint64_t *first, uint64_t *count);
/* Grouped PFADD across ranks, routed to the owners (C5 across GPUs; the
 * alternative to adding every pair locally and rsk_hll_reducescatter_pool).
 * Collective: every rank passes its own pairs -- 16-byte keys (16-byte
 * aligned) and uint32 group ids, both in device memory (n may be 0).  Each
 * pair is hashed where it lives and its 8-byte record (sketch, register index
 * and rank) shipped with grouped ncclSend/ncclRecv to the rank owning the
 * sketch (ownership as in rsk_hll_reducescatter_pool); every rank applies the
 * records it receives to its owned sketches [*first, *first + *count) only.
 * Afterwards those hold the registers one process would hold after adding
 * every rank's pairs (group ids >= the pool size are ignored); the rows
 * outside are not written (fetch them with rsk_hll_fetch_rows).  A pending
 * rsk_hll_clear is completed on the owned rows.  flags: RSK_FETCH_SELF also
 * routes this rank's own records through RCCL (the exchange on one GPU).
 * Argument errors on any rank are agreed on before anything moves. */
int rsk_hll_add_grouped_routed(rsk_hll *h, const rsk_keys *keys, const uint32_t *groups, uint32_t flags,
                               uint64_t *first, uint64_t *count);
/* Collective (every rank calls it, n may be 0): after a reduce-scatter, make
 * the local rows ids[0..n) equal to their owners' rows, so that
 * rsk_hll_count_union_batch / rsk_hll_merge_batch can read sketches owned by
 * other ranks (countWith/mergeWith across owners, RedissonHyperLogLog.java:
 * 83-97).  Ownership as in rsk_hll_reducescatter_pool; ids this rank owns are
 * skipped, duplicates fetched once.  Plan: counts then ids exchanged with
 * grouped ncclSend/ncclRecv, owners gather the rows into one staging buffer,
 * rows sent back and scattered into the pool.  The fetched rows are a
 * snapshot (caches invalidated); writes to them stay local. */
int rsk_hll_fetch_rows(rsk_hll *h, const uint64_t *ids, uint64_t n);
/* rsk_hll_fetch_rows with flags.  RSK_FETCH_SELF also routes the ids this rank
 * owns through the exchange (the rank gathers, sends to itself, receives and
 * scatters them): a no-op on the data that runs every exchange kernel on one
 * GPU (tests).  Argument errors on any rank (an id outside the pool) are
 * agreed on by all ranks before any row moves: every rank returns
 * RSK_ERR_INVALID_ARG and no rank is left waiting in a collective. */
#define RSK_FETCH_SELF 1u
int rsk_hll_fetch_rows_flags(rsk_hll *h, const uint64_t *ids, uint64_t n, uint32_t flags);
/* Bloom bit string := OR over all ranks (the node-level insert of sharded
 * keys, RedissonBloomFilter.java:80-114, before the replicated contains()).
 * RCCL has no bitwise-OR reduction: rank j owns a 1/N slice of the words;
 * grouped ncclSend/ncclRecv bring every rank's copy of slice j to rank j,
 * which ORs them into its filter, and send the merged slice back to every
 * rank -- straight out of and into the filter, one transfer per peer.  At
 * N = 1 nothing moves.  With RSK_FETCH_SELF the rank also exchanges its own
 * slice with itself (every step runs on one GPU; tests). */
int rsk_bloom_allreduce_or(rsk_bloom *b);
int rsk_bloom_allreduce_or_flags(rsk_bloom *b, uint32_t flags);

/* ------------------------------------------------------- exchange plans */
/* The host arithmetic the collectives above run (no GPU needed; exported so
 * the N > 1 plans are testable on CPU against redisson_amd/shard.py). */
/* Contiguous key-stream shard of rank `rank`: [*begin, *end). */
int rsk_plan_shard_range(uint64_t n, int world, int rank, uint64_t *begin, uint64_t *end);
/* Sketches owned after rsk_hll_reducescatter_pool. */
int rsk_plan_owned_range(uint64_t n, int nranks, int rank, uint64_t *first, uint64_t *count);
int rsk_plan_owner(uint64_t n, int nranks, uint64_t id, int *owner);
/* Words per rank of the Bloom slice-OR. */
int rsk_plan_bloom_slice_words(uint64_t nwords, int nranks, uint64_t *words);
/* rsk_hll_fetch_rows request plan: want_out (capacity n_ids) gets the
 * distinct requested ids ascending, counts_out[nranks] the rows asked of each
 * owner.  RSK_ERR_INVALID_ARG if an id is >= n. */
int rsk_plan_fetch(uint64_t n, int nranks, int rank, const uint64_t *ids, uint64_t n_ids, uint32_t flags,
                   uint64_t *want_out, uint64_t *n_want, uint64_t *counts_out);
/* rsk_hll_add_grouped_routed's traffic per owner: counts[s * G + g] = pairs of
 * group g on rank s; groups of >= heavy_min pairs owned by another rank (0:
 * none; at most heavy_cap per rank, lowest ids first) pre-combined at their
 * source into one 16 KiB row each.  Per rank (arrays of nranks): bytes received from the other ranks
 * (8 per light record, 16388 per heavy row with its id), heavy rows received,
 * light records its apply folds. */
int rsk_plan_route_recv(const uint64_t *counts, uint64_t G, int nranks, uint64_t heavy_min, uint64_t heavy_cap,
                        uint64_t *recv_bytes, uint64_t *recv_rows, uint64_t *apply_records);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif
#endif /* RSKETCH_H */
