/*
 * rsketch_diag.h -- benchmark and test support, exported by a library of its
 * own, librsketch_diag.so (the product library librsketch.so exports only
 * include/rsketch.h): memory-system microbenchmarks, kernel tuning variants,
 * the synthetic input streams of SURVEY.md 8d generated on the device, and
 * the route overrides tests use to force every pipeline of the library.
 * bench.py, scripts/ and tests/ use it.  Errors: rsk_diag_last_error().
 */
#ifndef RSKETCH_DIAG_H
#define RSKETCH_DIAG_H
#include "rsketch.h"

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

const char *rsk_diag_last_error(void);

/* Route override of a context (the product library has no other knob):
 *   bloom_stream  slice-routed insert: 0 auto, 1 at any batch size, -1 never
 *   bloom_part    exact-offset insert: 0 auto, 1 at any batch size, -1 never
 *   bloom_chunk   probes per chunk of the slice-routed insert (0 = default)
 *   sa_tiny       1: sub-regions of 32 probes (forces the overflow fallbacks)
 *   sa_kc         -1: the insert's sa1 with the runtime k also at k = 7 (0: a k = 7 instance)
 *   sa_v          the insert's sa2h tile: uint4 loads per lane, 0 (= 3), 6 or 8
 *   sa_dbg        TIMING ONLY (wrong filter): the insert's sa1 stores each tile's image
 *                 contiguously and the insert stops after sa1
 *   sa_full       -1: the insert's sa1 and the replies' rp1 without their branch-free path for
 *                 full super-tiles at k = 7
 *   sa_hash       TIMING ONLY (wrong filter): the insert's sa1 at k = 7 with the key words as
 *                 its hashes (1), also without the two mods (2)
 *   sa_parts      sa2 / rp2 parts per coarse bin (0 = default)
 *   reply         add() replies: 0 auto, 1 group-tag pipeline at any size, -1 sort path
 *   reply_chunk   probes per chunk of the group-tag pipeline (0 = default)
 *   reply_u       rp_treply keys (gather chains) per lane: 0 (= 2), 1, 2, 4
 *   reply_v       rp2 tile: uint4 loads per lane, 0 (= 8), 3 or 6
 *   reply_s       rp_tapply: wave steps whose segment loads are issued together, 0 (= 2), 1, 4
 *   reply_bal     rp_tapply: 0 an equal slice of the bucket's tiles per wave, -1 strided (A/B)
 *   reply_dbg     TIMING ONLY (wrong replies and T): rp_tapply without its
 *                 folds (bit 0) / without its T stores (bit 1)
 *   gpart         partitioned grouped PFADD: 0 auto, 1 any size, -1 never
 *   gpart_tm      1 (default): its first pass tile-major (hll_gpart1t), 0: exact-offset runs (hll_gcount + hll_gpart1)
 *   gapply_st     the grouped apply's row stores: 0 nontemporal (default), 1 plain, 2 none (TIMING ONLY)
 *   gpart_rt      the fine-bin sort's round: 0 8192 records (default), 1 16384 (one
 *                 workgroup per CU)
 *   io_trace      1: the batched export / import print their host phase times to stderr
 *   io_piece      batched export's copy-out pieces in MiB (0: 16)
 *   io_drain      batched export: 1 = each chunk's copy-out finished before the next chunk (A/B)
 *   copy_nt       staged host copies (host keys, export / import strings): 0 streaming stores, -1 memcpy (A/B)
 *   io_pin        batched export: 0 pin a pageable output buffer >= 256 MiB for the call, -1 never (staged)
 *   gpart_tile    tile-major first pass: 0 (default) 8192-record tiles, 1 16384 (one 512-lane block per CU)
 *   route_vranks  TEST ONLY, 1-rank communicator: rsk_hll_add_grouped_routed plans as rank route_vrank of
 *   route_vrank   route_vranks (its owned sub-range; records for the other owners are dropped)
 *   route_heavy   routed add's heavy-group pre-combine: 0 auto, -1 never, > 0 at any size with that many
 *                 pairs (estimated from a sample) making a group heavy
 *   gpart_poison  1: its fine-bin output is filled with 0xFF before the fine-bin pass (a slot the pass
 *                 leaves unwritten then corrupts a register: the tests' hole check)
 *   gpart_dbg     TIMING ONLY (the grouped add stops before its apply): bit 0 the fine-bin pass
 *                 stores each round's image contiguously, bit 1 no fine-bin count pass
 *   reset         every route back to automatic
 * Every route but sa_dbg, sa_hash, gpart_dbg and reply_dbg gives bit-identical results; they differ in speed only. */
int rsk_diag_set_route(rsk_ctx *ctx, const char *name, int64_t value);

/* add()-with-replies counters of a context since it was created: key groups
 * whose pending probes (a bit probed more than once by the group that probed
 * it first) were resolved in LDS, and chunks answered by the sort-path
 * fallback (a group's pending probes overflowed its LDS tables). */
int rsk_diag_reply_stats(rsk_ctx *ctx, uint64_t *pending_groups, uint64_t *fallbacks);

/* The SDMA engine the batched export's device->host copies (to_host = 1) or
 * the batched import's host->device copies (to_host = 0) use on this context
 * (-2: not measured yet, no export / import so far; -1: HIP's own copies) and
 * the rate measured in that direction on each of engines 0..7 (GB/s; 0: not
 * measured or not available). */
int rsk_diag_copy_engine(rsk_ctx *ctx, int to_host, int *engine, float *rates);

/* Marks a context dead, as a device error on one of its streams does: every
 * later call but rsk_shutdown fails with RSK_ERR_DEVICE (tests of the
 * bindings' release paths). */
int rsk_diag_mark_dead(rsk_ctx *ctx);

/* --------------------------------------------------------- diagnostics */
/* Memory-system microbenchmark on a device buffer (roofline denominators):
 * mode 0 stream read, 1 random 4 B gathers, 2 random 4 B atomicOr,
 * 3 stream copy (buffer halves), 4 stream write, 5 stream write with
 * nontemporal stores, 6 scattered segment reads of n_ops (256, 512 or 1024)
 * bytes, one uint4 per lane, every byte of the largest power-of-two number
 * of segments that fits read once (FETCH_SIZE calibration), 7 stream copy
 * (buffer halves) with the loads and the stores in different waves, 8 stream
 * read with 4 B per lane, 9 scattered segment reads of n_ops (128 or 256)
 * bytes, one dword per lane (FETCH_SIZE calibration of 4-byte loads).
 * *ms = device time of the one launch. */
int rsk_diag_membench(rsk_ctx *ctx, int mode, void *dev_buf, uint64_t bytes, uint64_t n_ops, double *ms);

/* Self send/recv of `bytes` (a multiple of 8) of a known pattern through the context's 1-rank
 * communicator, then a device compare (rsk_diag_p2p.hip): mode 0 one ncclSend/ncclRecv of bytes
 * ncclUint8 elements, mode 1 one of bytes/8 ncclUint64 elements, mode 2 pieces of <= 1 GiB
 * (the library's p2p_pieces).  bad_words: 4-byte words that differ; first_bad: the lowest one
 * (~0 if none). */
int rsk_diag_p2p_probe(rsk_ctx *ctx, uint64_t bytes, int mode, uint64_t *bad_words, uint64_t *first_bad);
/* Time one launch of a tuning variant of the 16-byte PFADD kernel (slabs only). */
int rsk_diag_hll_variant(rsk_ctx *ctx, int variant, const void *dev_keys16, uint64_t n, double *ms);
/* Time one launch of a variant of the blob+offsets PFADD kernel (slabs only):
 * 0 production (step-count sort, 1 key per lane), 1 sorted with 2 keys per lane,
 * 2 round-1 form (no prefetch, no sort), 3 sorted with 4 keys per lane. */
int rsk_diag_hll_var_variant(rsk_ctx *ctx, int variant, const void *dev_data, const uint64_t *dev_offsets, uint64_t n,
                             double *ms);
/* Time one launch of a tuning variant of the 16-byte Bloom contains kernel. */
int rsk_diag_bloom_contains_variant(rsk_ctx *ctx, int variant, rsk_bloom *b, const void *dev_keys16, uint64_t n,
                                    uint8_t *dev_out, double *ms);
/* Run the production 16-byte contains kernel's gather sequence with a tally:
 * replies into dev_out, *probes = bit gathers issued (early exit included). */
int rsk_diag_bloom_contains_probes(rsk_ctx *ctx, rsk_bloom *b, const void *dev_keys16, uint64_t n, uint8_t *dev_out,
                                   uint64_t *probes);

/* ----------------------------------------------- synthetic input streams */
/* SURVEY 8d generators, run on the device into caller-provided device
 * buffers (bench and parity tests; outside the timed region). */
int rsk_gen_keys16(rsk_ctx *ctx, uint64_t seed, uint64_t start, uint64_t n, void *dev_out);
int rsk_gen_grouped(rsk_ctx *ctx, uint64_t seed, uint64_t G, uint64_t start, uint64_t n, uint32_t *dev_groups,
                    void *dev_keys);
/* C5 Zipf(s) stress variant: group = Zipf(s) rank over [0, G) (rank 1 -> group 0)
 * drawn from splitmix64(seed + 3i) >> 1 against a u63 cumulative-weight table;
 * keys as rsk_gen_grouped (oracle: orc_gen_grouped_zipf). */
int rsk_gen_grouped_zipf(rsk_ctx *ctx, uint64_t seed, uint64_t G, double s, uint64_t start, uint64_t n,
                         uint32_t *dev_groups, void *dev_keys);
int rsk_gen_queries16(rsk_ctx *ctx, uint64_t qseed, uint64_t iseed, uint64_t n_ins, uint64_t start, uint64_t n,
                      void *dev_out);
/* Variable-length keys: lengths first (dev_offsets gets n+1 offsets), then
 * bytes into dev_blob (capacity blob_cap). */
int rsk_gen_varlen(rsk_ctx *ctx, uint64_t seed, uint64_t start, uint64_t n, uint64_t *dev_offsets, void *dev_blob,
                   uint64_t blob_cap, uint64_t *total_bytes);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif
#endif /* RSKETCH_DIAG_H */
