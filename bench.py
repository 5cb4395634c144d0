"""Benchmark: HLL addAll of 16-byte keys (+ count) on MI355X, BASELINE configs[1].

Step = RHyperLogLog.addAll(n synthetic 16-byte keys already resident in HBM)
       + (N > 1) RCCL MAX all-reduce of the 16384 registers + count().
The keys are the SURVEY.md 8d C2 stream (splitmix64, seed 0x5EED0002), each
rank taking its own contiguous range (weak scaling: n keys per GPU).
Secondary fields of the same line:
  `bloom`   the C3 Bloom filter per node (1B inserts at 1% FPP, EXTENDED mode,
            sharded over the ranks and merged with the RCCL slice-OR, then 1B
            contains queries sharded over the replicated filter);
  `c4`      BASELINE configs[3] per GPU: 1B variable-length keys (+ RCCL MAX);
  `c5`, `c5_zipf`  BASELINE configs[4] per GPU: 1M sketches, 500M pairs per
            step, uniform and Zipf(1.1) groups, with count / countWith / mergeWith;
each with its own ms_per_step, roofline and PMC traffic (--no-extra skips them).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--keys N_PER_GPU]
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SEED_C2, SEED_C3, SEED_Q, SEED_C4, SEED_C5 = 0x5EED0002, 0x5EED0003, 0x5EED0004, 0x5EED0005, 0x5EED0006


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kernel: str, config: dict):
    """HBM bytes per launch from a committed rocprofv3 PMC summary taken with
    this same bench configuration (null if none matches)."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("config") != config:
            continue
        k = d.get("kernels", {}).get(kernel)
        if k and k.get("hbm_bytes_per_launch"):
            best = {"bytes": k["hbm_bytes_per_launch"], "source": os.path.relpath(p, ROOT),
                    "note": k.get("hbm_bytes_note")}
    return best


def pcie_inclusive(client, keys_host):
    """PFADD of host-resident keys (pageable numpy, the JNI direct-buffer case):
    the staging copies over PCIe are inside the timed region.  Never `value`."""
    from redisson_amd import KeyBatch

    hll = client.getHyperLogLog("bench-pcie")
    kb = KeyBatch.from_numpy(keys_host.reshape(-1, 16))
    hll.addAll(kb)  # warm-up (staging buffer allocation)
    t0 = time.perf_counter()
    hll.addAll(kb)
    dt = time.perf_counter() - t0
    n = kb.n
    return {"value": n / dt, "unit": "keys/s", "GBps_host_to_hbm": 16 * n / dt / 1e9,
            "sample": "%d C2 16-byte keys in pageable host memory, one addAll (256 MiB chunks through two pinned host stages)" % n}


def cpu_baseline(sample_keys: int, passes: int, threads: int):
    """The oracle's restatement of Redis PFADD (hllPatLen + register max) over
    a pre-generated in-memory sample of the same C2 stream: one core (the
    Redis-equivalent, Redis being single-threaded) as `value`, and all of the
    host cores this job may use (OpenMP, private registers + max-merge)."""
    import numpy as np

    from oracle import oracle as O

    keys = O.gen_keys16(SEED_C2, 0, sample_keys)
    regs = np.zeros(O.REGISTERS, np.uint8)
    t0 = time.perf_counter()
    for _ in range(passes):
        O.hll_add(regs, keys, None, 16, sample_keys)
    dt = time.perf_counter() - t0
    mt = np.zeros(O.REGISTERS, np.uint8)
    t1 = time.perf_counter()
    for _ in range(passes):
        O.hll_add_fixed_mt(mt, keys, 16, sample_keys, threads)
    dt_mt = time.perf_counter() - t1
    assert np.array_equal(mt, regs)
    return {"value": sample_keys * passes / dt, "unit": "keys/s", "cores": 1, "kind": "port",
            "sample": "%d passes over %d C2 16-byte keys (%.1f s, oracle/rsk_oracle.c orc_hll_add_raw, "
                      "Redis 3.2.0 PFADD arithmetic, 1 thread)" % (passes, sample_keys, dt),
            "all_cores": {"value": sample_keys * passes / dt_mt, "unit": "keys/s", "cores": threads,
                          "sample": "same sample, orc_hll_add_fixed_mt, %d OpenMP threads (%.1f s)"
                                    % (threads, dt_mt)}}


def bloom_cpu_baseline(n_ins: int, sample_1t: int, sample_mt: int, threads: int):
    """BASELINE.md's Bloom CPU restatement: inserts into the filter sized for
    n_ins @1% FPP (3,834,023,350 bits, k=7 at 4e8), the reference's own hash
    scheme (xx_r39 + farmUo, u63 mod) and SETBIT addressing, from the oracle."""
    import numpy as np

    from oracle import oracle as O

    size = O.bloom_optimal_bits(n_ins, 0.01)
    k = O.bloom_optimal_k(n_ins, size)
    bits = np.zeros((size + 7) // 8, np.uint8)
    keys = O.gen_keys16(SEED_C3, 0, sample_1t)
    t0 = time.perf_counter()
    O.bloom_add_batch(bits, size, k, keys, None, 16, sample_1t, want=False)
    dt = time.perf_counter() - t0
    del keys
    t1 = time.perf_counter()
    O.bloom_add_gen16_mt(bits, size, k, SEED_C3, sample_1t, sample_mt, threads)
    dt_mt = time.perf_counter() - t1
    return {"value": sample_1t / dt, "unit": "keys/s", "cores": 1, "kind": "port",
            "sample": "%d C3 16-byte keys (pre-generated, %.1f s) inserted into a %d-bit filter (k=%d: %d inserts "
                      "@1%% FPP, BASELINE.md), oracle orc_bloom_add_batch, 1 thread" % (sample_1t, dt, size, k, n_ins),
            "all_cores": {"value": sample_mt / dt_mt, "unit": "keys/s", "cores": threads,
                          "sample": "the next %d keys of the stream, orc_bloom_add_gen16_mt (keys generated inline), "
                                    "%d OpenMP threads (%.1f s)" % (sample_mt, threads, dt_mt)}}


def random_access_peaks(engine, nbytes: int, reps: int = 3):
    """Live random-access denominators over a buffer the size of the filter:
    4-byte gathers and 4-byte atomicOr at uniformly random words (rsk_diag_membench)."""
    from redisson_amd import _lib, devmem

    D = _lib.diag()
    buf = devmem.DeviceBuffer(engine, nbytes)
    buf.zero()
    ops = 1 << 30
    best = {}
    for name, mode in (("gather4B", 1), ("atomicor4B", 2)):
        for _ in range(reps):
            ms = ctypes.c_double()
            _lib.check_diag(D.rsk_diag_membench(engine.ctx, mode, buf.ptr, nbytes, ops, ctypes.byref(ms)))
            best[name] = max(best.get(name, 0.0), ops / (ms.value / 1e3))
    buf.free()
    return best


def bloom_bench(engine, n_ins: int, n_q: int, reps: int, rank: int = 0, world: int = 1, with_replies: bool = True,
                keep_bits: bool = False):
    """Node-level Bloom (BASELINE configs[2]; north_star "Bloom lookups/s (node)",
    SURVEY 8e): the C3 stream's n_ins inserts are sharded over the ranks, each
    rank inserts its shard into its own filter of the full size, the partial bit
    strings are merged by rsk_bloom_allreduce_or (slices to their owners, OR,
    merged slices back over RCCL; at N = 1 the same call moves nothing), and
    each rank answers its 1/N of the n_q queries against the replicated filter.
    Phase times are the max over ranks; a phase ends on every rank's device."""
    import numpy as np

    from redisson_amd import _lib, devmem, shard

    L = _lib.load()
    size = ctypes.c_int64()
    k = ctypes.c_int32()
    _lib.check(L.rsk_bloom_params(n_ins, 0.01, _lib.RSK_BLOOM_EXTENDED, ctypes.byref(size), ctypes.byref(k)))
    ilo, ihi = shard.ShardPlan(n_ins, world).range(rank)
    qlo, qhi = shard.ShardPlan(n_q, world).range(rank)
    m_ins, m_q = ihi - ilo, qhi - qlo
    ins = devmem.gen_keys16(engine, SEED_C3, ilo, m_ins)
    qs = devmem.gen_queries16(engine, SEED_Q, SEED_C3, n_ins, qlo, m_q)
    out = devmem.DeviceBuffer(engine, max(1, m_q))
    ki = ins.keys_fixed(m_ins, 16).as_struct()
    kq = qs.keys_fixed(m_q, 16).as_struct()

    def node_max(vals, op="max"):
        if world == 1:
            return list(vals)
        import torch
        import torch.distributed as dist

        t = torch.tensor(list(vals), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return t.tolist()

    def barrier():
        engine.sync()
        if world > 1:
            import torch.distributed as dist

            dist.barrier()

    phases = []
    hits = probes = 0
    bits = None
    for r in range(reps + 1):
        if r == 1:  # rep 0 is warm-up (first-call scratch allocation); kernel times from rep 1
            engine.prof_reset()
            engine.prof_enable(True)
        b = ctypes.c_void_p()
        _lib.check(L.rsk_bloom_create(engine.ctx, size.value, k.value, ctypes.byref(b)))
        barrier()
        t0 = time.perf_counter()
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ki), None))
        engine.sync()
        t1 = time.perf_counter()
        shard.bloom_allreduce_or(b)  # returns once this rank's filter is the node's
        t2 = time.perf_counter()
        _lib.check(L.rsk_bloom_contains(b, ctypes.byref(kq), out.ptr))
        engine.sync()
        t3 = time.perf_counter()
        if r:
            phases.append((t1 - t0, t2 - t1, t2 - t0, t3 - t2))
        if r == reps:
            hits = int(out.to_numpy()[:m_q].sum())
            # untimed: the gathers the contains kernel issues for these queries
            pr = ctypes.c_uint64()
            _lib.check_diag(_lib.diag().rsk_diag_bloom_contains_probes(engine.ctx, b, qs.ptr, m_q, out.ptr,
                                                                       ctypes.byref(pr)))
            probes = pr.value
            bc = ctypes.c_uint64()
            _lib.check(L.rsk_bloom_bitcount(b, ctypes.byref(bc)))
            fill = bc.value / size.value
            if keep_bits:
                bits = np.zeros((size.value + 7) // 8, np.uint8)
                n_ = ctypes.c_size_t()
                _lib.check(L.rsk_bloom_export_bits(b, bits.ctypes.data, bits.size, ctypes.byref(n_)))
        L.rsk_bloom_destroy(b)
        barrier()
    engine.prof_enable(False)
    # per rep: the slowest rank's phase; then the best rep
    per_rep = [node_max(p) for p in phases]
    ins_local_s = min(p[0] for p in per_rep)
    merge_s = min(p[1] for p in per_rep)
    add_s = min(p[2] for p in per_rep)
    con_s = min(p[3] for p in per_rep)
    hits, probes = (int(v) for v in node_max([hits, probes], "sum"))
    add_ms, add_n = engine.prof_read("bloom_add16")
    con_ms, con_n = engine.prof_read("bloom_contains16")
    stages = {}
    for name in ("bloom_st1", "bloom_st_mid", "bloom_st2", "bloom_st_apply",
                 "bloom_part_hist", "bloom_part1", "bloom_part2", "bloom_slice_apply"):
        ms, cnt = engine.prof_read(name)
        if cnt:
            stages[name] = ms / max(1, add_n)  # per insert batch (summed over its chunks)
    replies = None
    if with_replies and world == 1:
        # RBloomFilter.add's per-element reply (RedissonBloomFilter.java:100-107) for
        # every key of the batch, in input order, into a fresh filter: run 0 warms
        # up (the pipeline's scratch is allocated), run 1 is timed.
        rout = devmem.DeviceBuffer(engine, n_ins)
        for r in range(2):
            if r == 1:
                engine.prof_reset()
                engine.prof_enable(True)
            b = ctypes.c_void_p()
            _lib.check(L.rsk_bloom_create(engine.ctx, size.value, k.value, ctypes.byref(b)))
            engine.sync()
            t0 = time.perf_counter()
            _lib.check(L.rsk_bloom_add(b, ctypes.byref(ki), rout.ptr))
            engine.sync()
            dt = time.perf_counter() - t0
            L.rsk_bloom_destroy(b)
        engine.prof_enable(False)
        rstages = {}
        for name in ("bloom_rp1", "bloom_rp_mid", "bloom_rp2", "bloom_rp_apply", "bloom_rp_reply", "bloom_rp_fallback"):
            ms, cnt = engine.prof_read(name)
            if cnt:
                rstages[name] = ms
        chunks = -(-n_ins * k.value // (1 << 33))  # rsk_bloom_reply.hip: chunks of <= 2^33 probes
        # per probe: 4 B record written by rp1, read + written by rp2, read by
        # rp_tapply; per chunk: the group-tag table T (2 B per filter bit) written,
        # the filter read and written; keys read by rp1 and by the reply pass
        model = n_ins * k.value * 16 + chunks * (2 * size.value + 2 * (size.value // 8)) + 32 * n_ins
        replies = {"keys": n_ins, "ms": dt * 1e3, "keys_per_s": n_ins / dt,
                   "replies_true": int(rout.to_numpy().sum()), "stage_ms": rstages, "chunks": chunks,
                   "traffic_model_GB": model / 1e9, "model_GBps": model / dt / 1e9,
                   "model_frac_of_8TBps": model / dt / 8e12,
                   "note": "rsk_bloom_add with added_out (sequential SETBIT-reply semantics), fresh filter, "
                           "partitioned group-tag pipeline (rsk_bloom_reply.hip); model excludes the reply "
                           "pass's random gathers"}
        tr = pmc_traffic("bloom_add_replies", {"workload": "bloom_add_replies", "keys": n_ins, "zipf": 0.0,
                                               "bloom_keys": n_ins})
        if tr:  # the same pipeline alone under rocprofv3 (scripts/reply_profile.py)
            replies["traffic"] = tr["bytes"]
            replies["traffic_source"] = tr["source"]
            replies["traffic_GBps"] = tr["bytes"] / dt / 1e9
        rout.free()
    for buf in (ins, qs, out):
        buf.free()
    peaks = random_access_peaks(engine, (size.value + 7) // 8)
    gathers_per_s = probes / con_s
    sets_per_s = n_ins * k.value / add_s
    res = {"config": "C3: %d inserts @1%% FPP (size %d bits, k=%d, EXTENDED), %d contains (50%% inserted); "
                     "%d rank(s): inserts and queries sharded, filters merged by rsk_bloom_allreduce_or"
                     % (n_ins, size.value, k.value, n_q, world),
            "n_gpus": world, "path": "node: sharded insert + rsk_bloom_allreduce_or + sharded contains",
            "insert_keys_per_s": n_ins / add_s, "contains_keys_per_s": n_q / con_s,
            "insert_ms": add_s * 1e3, "insert_local_ms": ins_local_s * 1e3, "merge_ms": merge_s * 1e3,
            "contains_ms": con_s * 1e3, "contains_true": hits,
            "insert_kernel_avg_ms": add_ms / max(1, add_n), "contains_kernel_avg_ms": con_ms / max(1, con_n),
            "insert_stage_ms": stages,
            "insert_bit_rmw_per_s": sets_per_s,
            "contains_probe_gathers_per_s": gathers_per_s,
            "random_access_roofline": {
                "filter_fill": fill,
                "contains": {"bound": "random 4 B gather", "gathers_issued": probes,
                             "gathers_per_key": probes / n_q, "achieved": gathers_per_s,
                             "peak": peaks["gather4B"], "unit": "gathers/s",
                             "frac": gathers_per_s / peaks["gather4B"],
                             "hbm_GBps_at_64B_per_gather": gathers_per_s * 64 / 1e9},
                "insert": {"bound": "random 4 B atomicOr (direct kernel)", "achieved": sets_per_s,
                           "peak": peaks["atomicor4B"], "unit": "bit-sets/s",
                           "ratio": sets_per_s / peaks["atomicor4B"],
                           "note": "slice-partitioned: probes sorted into 64 KiB LDS-resident filter slices, "
                                   "so the insert is not bound by memory-side atomics"},
                "peaks_measured_on": "a zeroed buffer of the filter's size, 2^30 uniformly random ops, best of 3"},
            "insert_roofline": insert_roofline(n_ins // world, k.value, size.value, ins_local_s),
            "insert_with_replies": replies}
    if keep_bits:
        res["bits"] = bits
    return res


def insert_roofline(n: int, k: int, size: int, secs: float):
    """HBM view of the C3 insert: the streaming floor (every key read once, the
    filter read and written once) and the append pipeline's own traffic model
    (sa1 writes 4 B per probe, sa2h reads them and writes 2 B records, apply
    reads those: 12 B per probe), both as bytes / measured insert time."""
    filt = (size + 7) // 8
    floor_b = 16.0 * n + 2.0 * filt
    model_b = 16.0 * n + 12.0 * k * n + 2.0 * filt
    return {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
            "algorithmic_bytes": floor_b, "achieved": floor_b / secs / 1e9,
            "frac": floor_b / secs / 1e9 / HBM_PEAK_GBS,
            "pipeline_model_bytes": model_b, "pipeline_model_GBps": model_b / secs / 1e9,
            "pipeline_model_frac": model_b / secs / 1e9 / HBM_PEAK_GBS}


WORKLOADS = {
    "c2": "HLL addAll of 16-byte keys + count() (BASELINE configs[1])",
    "c4": "HLL addAll of variable-length string keys (8-64 B, blob+offsets) + count() (BASELINE configs[3])",
    "c5": "Grouped HLL: %d sketches cleared each step, grouped add + count(all) + %d countWith + %d mergeWith "
          "(BASELINE configs[4]), issued as one pipelined batch per step (the library's async calls, one wait); "
          "N > 1: each rank's pairs hashed locally and routed to the rank owning their sketch "
          "(rsk_hll_add_grouped_routed: 8-byte records over RCCL send/recv), each rank counting its "
          "own 1/N of the sketches and running countWith/mergeWith led by them against partners from "
          "all G, fetched from their owners over RCCL",
}


def run_hll(ctx, wl: str, n: int, steps: int, warmup: int, zipf: float = 0.0, groups_n: int = 1_000_000,
            batch_ops: int = 100_000, bloom_keys: int = 0):
    """One HLL workload (c2 / c4 / c5) on this rank: inputs generated into HBM
    (untimed), `warmup` untimed steps, then `steps` timed steps between
    barriers; the max over ranks of the elapsed time.  Returns the bench
    fields of that workload (value, ms_per_step, roofline, ...)."""
    engine, client, rank, world = ctx["engine"], ctx["client"], ctx["rank"], ctx["world"]
    from redisson_amd import devmem, shard

    extra = {}
    hll = client.getHyperLogLog("bench-" + wl)
    if wl == "c2":
        keys = devmem.gen_keys16(engine, SEED_C2, rank * n, n)
        kb = keys.keys_fixed(n, 16)
        kern, unit_bytes = "hll_add16", 16.0 * n
        bufs = [keys]
    elif wl == "c4":
        blob, offs, tot = devmem.gen_varlen(engine, SEED_C4, rank * n, n)
        kb = blob.keys_var(offs, n)
        kern, unit_bytes = "hll_add_var", float(tot + 8 * n)
        extra = {"key_bytes_total": tot, "mean_key_len": tot / n}
        bufs = [blob, offs]
    else:  # c5: grouped COUNT DISTINCT
        from redisson_amd.hyperloglog import GroupedHyperLogLog
        import numpy as np

        G = groups_n
        if zipf > 0:
            groups, gkeys = devmem.gen_grouped_zipf(engine, SEED_C5, G, zipf, rank * n, n)
            extra = {"group_distribution": "Zipf(%g) over the %d sketches (rank 1 = sketch 0)" % (zipf, G)}
        else:
            groups, gkeys = devmem.gen_grouped(engine, SEED_C5, G, rank * n, n)
        kb = gkeys.keys_fixed(n, 16)
        pool = GroupedHyperLogLog(engine, G)
        # N > 1: the pairs are routed to their owners, rank r owns a contiguous 1/N
        # of the sketches and counts those; countWith(a, b) runs on a's owner and
        # mergeWith(dst, src) on dst's owner, with b / src drawn from all G
        # sketches and fetched from their owners (rsk_hll_fetch_rows, RCCL).
        own_first, own_count = shard.owned_range(G, world, rank)
        own_ids = np.arange(own_first, own_first + own_count, dtype=np.uint64)
        rng = np.random.default_rng(5 + rank)
        cw = np.stack([rng.integers(own_first, own_first + own_count, size=batch_ops, dtype=np.uint64),
                       rng.integers(0, G, size=batch_ops, dtype=np.uint64)], 1)
        md = rng.integers(own_first, own_first + own_count, size=batch_ops, dtype=np.uint64)
        ms_ = rng.integers(0, G, size=batch_ops, dtype=np.uint64)
        remote = np.concatenate([cw[:, 1], ms_])
        kern, unit_bytes = "hll_add_grouped16", 20.0 * n
        bufs = [groups, gkeys]
        counts_out = np.empty(max(G, own_count), np.uint64)  # the caller's reply buffers, reused across steps
        cw_out = np.empty(batch_ops, np.uint64)

    def step():
        if wl == "c5":
            # One pipelined batch per step (the async calls, ordered on the
            # context stream; RBatch-style): the host work of each call
            # overlaps the GPU work queued before it, one wait at the end.
            pool.clear()  # every step builds the G sketches from empty (fresh PFADDs, not idempotent re-adds)
            if world > 1:
                # pairs hashed here, 8-byte records sent to the rank owning their
                # sketch (grouped ncclSend/ncclRecv), applied to the owned rows only
                assert shard.hll_add_grouped_routed(pool.pool, kb, groups) == (own_first, own_count)
                ops = [pool.count_async(counts_out, own_ids)]
                ops[0].wait()
                shard.hll_fetch_rows(pool.pool, remote)  # partner / source rows from their owners
                ops = []
            else:
                ops = [pool.add_async(kb, groups), pool.count_async(counts_out)]
            ops.append(pool.countWith_async(cw, cw_out))
            ops.append(pool.mergeWith_async(md, ms_))
            for op in ops:
                op.wait()
            return int(counts_out[0])
        hll.addAll(kb)
        if world > 1:
            slot = client._hll_slot("bench-" + wl, False)
            shard.hll_allreduce(slot.pool, slot.id)  # RCCL MAX over xGMI
        return hll.count()

    for _ in range(warmup):
        step()

    def barrier():
        engine.sync()
        if world > 1:
            import torch.distributed as dist

            dist.barrier()

    engine.prof_reset()
    engine.prof_enable(True)
    barrier()
    cards = []
    t0 = time.perf_counter()
    for _ in range(steps):
        cards.append(step())
    barrier()
    elapsed = time.perf_counter() - t0
    cards_agree = None
    if world > 1 and wl != "c5":
        # after each step's RCCL MAX all-reduce every rank holds the same
        # registers, so every rank's count() of every step must agree
        import torch.distributed as dist

        everyone = [None] * world
        dist.all_gather_object(everyone, cards)
        cards_agree = all(c == cards for c in everyone)
        if not cards_agree:
            raise SystemExit("count() differs between ranks after the all-reduce: %r" % (everyone,))
    engine.prof_enable(False)
    add_ms, add_launches = engine.prof_read(kern)
    kern_label = kern + "_kernel"
    stage_ms = None
    if wl == "c5" and add_launches == 0:
        # the partitioned grouped PFADD (rsk_hll_group.hip): its stages together are the add
        stages = ("hll_gpart_count", "hll_gpart1", "hll_gpart2", "hll_gapply")
        reads = {st: engine.prof_read(st) for st in stages}
        add_launches = reads["hll_gapply"][1]
        add_ms = sum(v[0] for v in reads.values())
        stage_ms = {st: v[0] / max(1, v[1]) for st, v in reads.items()}
        kern_label = ("hll_add_grouped (partitioned, tile-major: hll_gpart1t, hll_hdr_transpose + scan, "
                      "hll_gparts_tm + hll_gcount2t + scan + hll_gfine + hll_gpart2t, hll_gapply)")
    red_ms, red_launches = engine.prof_read("hll_reduce")
    side = {name: engine.prof_read(name) for name in ("hll_count", "hll_union_count", "hll_merge",
                                                       "hll_allreduce", "hll_allreduce_pool",
                                                       "hll_reducescatter_pool", "hll_fetch_rows", "hll_clear")}
    if world > 1:
        import torch
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    value = n * world * steps / elapsed
    avg_launch_s = (add_ms / 1e3) / max(1, add_launches)
    achieved = unit_bytes / avg_launch_s / 1e9  # algorithmic bytes per launch / launch time
    res = {
        "value": value,
        "unit": "keys/s" if wl != "c5" else "pairs/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "config": dict({"workload": WORKLOADS[wl] % ((groups_n, batch_ops, batch_ops) if wl == "c5" else ()),
                        "keys_per_gpu": n, "global_keys_per_step": n * world,
                        "parallelism": ("pair-stream sharding, pairs routed to the sketch owners over RCCL"
                                        if wl == "c5" else
                                        "key-stream sharding, RCCL MAX all-reduce of the registers") if world > 1
                        else "single GPU", "redis_semantics": "3.2.0"}, **extra),
        "roofline": {"bound": "hbm", "kernel": kern_label, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None,
                     "avg_launch_ms": avg_launch_s * 1e3, "launches": add_launches,
                     "reduce_avg_ms": red_ms / max(1, red_launches),
                     "algorithmic_bytes_per_launch": unit_bytes},
        "side_kernels_ms_per_launch": {k: (v[0] / v[1] if v[1] else None) for k, v in side.items()},
        "count": int(cards[-1]),
    }
    if cards_agree is not None:
        res["count_identical_across_ranks_every_step"] = cards_agree
    pmc_cfg = {"workload": wl, "keys": n, "zipf": zipf, "bloom_keys": bloom_keys}
    tr = pmc_traffic("hll_add_grouped_partitioned" if stage_ms else kern + "_kernel", pmc_cfg)
    if tr:
        res["roofline"]["traffic"] = tr["bytes"]
        res["roofline"]["traffic_source"] = tr["source"]
        if tr.get("note"):
            res["roofline"]["traffic_note"] = tr["note"]
    if wl == "c5":
        # The grouped add must also write every touched sketch once whatever
        # the update order (16 KiB per touched sketch; at 500 pairs/sketch all
        # G are touched; the pool was just cleared, so nothing need be read):
        # the state-inclusive floor.
        touched = groups_n * -math.expm1(-n / groups_n)  # expected sketches hit by n uniform pairs
        if zipf > 0:  # expected sketches hit by n Zipf pairs: sum over ranks of 1 - (1 - p_r)^n
            import numpy as np

            w = np.arange(1, groups_n + 1, dtype=np.float64) ** -zipf
            touched = float(-np.expm1(n * np.log1p(-w / w.sum())).sum())
        state = 1.0 * touched * 16384  # written once; the cleared pool need not be read
        res["roofline"]["state_bytes_per_launch"] = state
        res["roofline"]["frac_incl_state"] = (unit_bytes + state) / avg_launch_s / 1e9 / HBM_PEAK_GBS
        if stage_ms:
            res["roofline"]["stage_ms_per_launch"] = stage_ms
        res["add_ms_per_step"] = avg_launch_s * 1e3
        if world == 1 and zipf == 0:
            res["checkpoint"] = checkpoint_bench(engine, pool)
    for b in bufs:
        b.free()
    if wl == "c5":
        pool.close()
    else:
        hll.delete()
    return res


def checkpoint_bench(engine, pool):
    """The pool's checkpoint (the export path is the checkpoint): GET
    of every sketch as its Redis string in one rsk_hll_export_redis_batch call
    into host memory, then SET of all of them into a fresh pool in one
    rsk_hll_import_redis_batch call; the restored pool re-exports to the same
    bytes.  Host memory at both ends (PCIe inclusive)."""
    import numpy as np

    from redisson_amd.hyperloglog import GroupedHyperLogLog

    ids = np.arange(pool.n, dtype=np.uint64)
    data, offs = pool.exportRedis(ids)  # warm-up: sizes the buffer (and touches its pages)
    t_exp = []
    for _ in range(3):
        t0 = time.perf_counter()
        data, offs = pool.exportRedis(ids, out=data)
        t_exp.append(time.perf_counter() - t0)
    lens = np.diff(offs.astype(np.int64))
    fresh = GroupedHyperLogLog(engine, pool.n)
    fresh.importRedis(ids, data, offs)  # warm-up (scratch)
    t_imp = []
    for _ in range(3):
        t0 = time.perf_counter()
        fresh.importRedis(ids, data, offs)
        t_imp.append(time.perf_counter() - t0)
    d2, o2 = fresh.exportRedis(ids, out=np.empty_like(data))
    same = bool(np.array_equal(o2, offs) and np.array_equal(d2, data))
    # the same calls with the host buffer registered once (rsk_host_register: a reused buffer,
    # e.g. a Java direct ByteBuffer): DMA straight to / from it, no pinned stage or host copy
    t0 = time.perf_counter()
    engine.host_register(data)
    t_reg = time.perf_counter() - t0
    r_exp, r_imp = [], []
    try:
        for _ in range(2):
            t0 = time.perf_counter()
            pool.exportRedis(ids, out=data)
            r_exp.append(time.perf_counter() - t0)
        for _ in range(2):
            t0 = time.perf_counter()
            fresh.importRedis(ids, data, offs)
            r_imp.append(time.perf_counter() - t0)
        d3, o3 = fresh.exportRedis(ids, out=np.empty_like(data))
        same = same and bool(np.array_equal(o3, offs) and np.array_equal(d3, d2))
    finally:
        engine.host_unregister(data)
    fresh.close()
    return {"sketches": int(pool.n), "bytes": int(offs[-1]), "sparse_keys": int((lens < 12304).sum()),
            "export_ms": min(t_exp) * 1e3, "import_ms": min(t_imp) * 1e3,
            "export_ms_each": [t * 1e3 for t in t_exp], "import_ms_each": [t * 1e3 for t in t_imp],
            "export_GBps": int(offs[-1]) / min(t_exp) / 1e9, "import_GBps": int(offs[-1]) / min(t_imp) / 1e9,
            "export_sketches_per_s": pool.n / min(t_exp), "import_sketches_per_s": pool.n / min(t_imp),
            "round_trip_identical": same,
            "registered_host_buffer": {"register_ms": t_reg * 1e3, "export_ms": min(r_exp) * 1e3,
                                       "import_ms": min(r_imp) * 1e3,
                                       "export_GBps": int(offs[-1]) / min(r_exp) / 1e9,
                                       "import_GBps": int(offs[-1]) / min(r_imp) / 1e9,
                                       "note": "the host buffer pinned once with rsk_host_register (not timed in "
                                               "export_ms / import_ms; register_ms is its one-time cost)"},
            "note": "rsk_hll_export_redis_batch / rsk_hll_import_redis_batch of every sketch after the timed "
                    "steps, pageable host buffers (PCIe inclusive; the export pins its >= 256 MiB output buffer "
                    "for the call, inside export_ms), one call each, best of 3 (all listed)"}


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` without a launcher around it (no WORLD_SIZE in the
    environment): start N fresh worker processes of this same command, one per
    GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as
    torch.distributed.run would set them, forward rank 0's JSON line, and fail
    if any worker fails.  This process makes no HIP, RCCL or torch call (it
    never touched the GPU, and it execs nothing): the workers own the devices.
    After the first worker fails the others are stopped (they would wait in a
    collective for the dead rank), by their own pids."""
    import signal
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True))
    # rank 0's stdout is drained by a thread so a full pipe never stalls it
    import threading

    out = []
    t = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    t.start()
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log("launcher: rank %d exited with %d; stopping the other ranks" % (r, code))
                for q in sorted(live):
                    try:
                        os.killpg(procs[q].pid, signal.SIGTERM)  # the worker's own session, started above
                    except ProcessLookupError:
                        pass
        time.sleep(0.05)
    t.join(timeout=30)
    text = out[0].decode() if out and out[0] else ""
    lines = [ln for ln in text.splitlines() if ln.startswith("{")]
    if rc == 0 and not lines:
        log("launcher: rank 0 printed no JSON line")
        rc = 1
    if lines:
        print(lines[-1], flush=True)
    return rc


def launcher_selftest(rank: int, world: int) -> None:
    """--launcher-selftest: the launch plumbing alone, stopped before
    librsketch is loaded -- every rank joins one gloo group and rank 0 prints
    the ranks that joined (tests/test_bench_launcher.py, on the CPU)."""
    if world == 1:
        print(json.dumps({"launcher_selftest": True, "n_gpus": 1, "ranks": [{"rank": 0, "local_rank": 0,
                                                                             "pid": os.getpid()}]}), flush=True)
        return
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    if os.environ.get("RSK_SELFTEST_FAIL_RANK") == str(rank):
        raise SystemExit(3)  # the test of a failing rank: the others then wait in all_gather until stopped
    everyone = [None] * world
    dist.all_gather_object(everyone, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                                      "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"launcher_selftest": True, "n_gpus": world, "ranks": everyone}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU; without a launcher (no WORLD_SIZE) bench.py starts them itself")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="test the multi-rank launch only: ranks join a gloo group and stop (no GPU)")
    # defaults: the kernel trace shows the first ~12 launches on a box running
    # slower while the clock settles (profiles/r02_roofline_check.json)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--workload", choices=("c2", "c4", "c5"), default="c2",
                    help="c2: 16-byte keys (headline); c4: variable-length keys; c5: grouped sketches")
    ap.add_argument("--keys", type=int, default=None,
                    help="keys (pairs for c5) per GPU; default 1e9 (c2, c4), 5e8 for c5 (4e9 pairs over 8 GPUs)")
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--zipf", type=float, default=0.0,
                    help="c5: draw groups Zipf(S) over the sketches (SURVEY 8d stress variant; 0 = uniform)")
    ap.add_argument("--batch-ops", type=int, default=100_000)
    ap.add_argument("--bloom-keys", type=int, default=1_000_000_000)
    ap.add_argument("--no-bloom", action="store_true")
    ap.add_argument("--no-bloom-replies", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="c2 only: skip the secondary C4 / C5 / C5-Zipf workloads (keys c4, c5, c5_zipf)")
    ap.add_argument("--extra-steps", type=int, default=20)
    ap.add_argument("--extra-warmup", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=128 << 20)
    ap.add_argument("--cpu-passes", type=int, default=8)
    ap.add_argument("--cpu-threads", type=int, default=16, help="all-cores CPU figure (the GPU box's CPU share is 16)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start the ranks here, before anything touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a silent N = 1 run reported as N GPUs (or the reverse) would corrupt the scaling curve
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus=%d; refusing to run" % (world, args.gpus))
    if args.launcher_selftest:
        launcher_selftest(rank, world)
        return

    # librsketch (system ROCm runtime) is loaded before torch is imported, so
    # the process has exactly one initialised HIP/HSA runtime.
    from redisson_amd import _lib as _early

    _early.load()
    # The bench support library (generators) too: loaded after torch, its HIP
    # calls bound to a runtime rocprofv3 had not hooked (a launch through a
    # null dispatch entry under --kernel-trace).
    _early.diag()
    import torch.distributed as dist

    if world > 1:
        # gloo only ships the RCCL id and the timings; the data path is RCCL.
        dist.init_process_group("gloo")

    from redisson_amd import devmem, shard
    from redisson_amd.client import Config, Redisson

    client = Redisson.create(Config(device=local))
    engine = client.engine
    if world > 1:
        shard.init_comm(engine)
    elif not args.no_bloom and args.workload == "c2":
        shard.init_comm_single(engine)  # the node-level Bloom merge runs through the same call at N = 1
    # what RCCL itself reports (ncclCommCount): every rank must have joined
    rccl_nranks, rccl_rank = shard.comm_info(engine)
    if world > 1 and (rccl_nranks, rccl_rank) != (world, rank):
        raise SystemExit("RCCL reports %d ranks (this one %d), WORLD_SIZE is %d (RANK %d)"
                         % (rccl_nranks, rccl_rank, world, rank))
    ctx = {"engine": engine, "client": client, "rank": rank, "world": world}
    wl = args.workload
    n = args.keys if args.keys is not None else (500_000_000 if wl == "c5" else 1_000_000_000)
    bloom_on = wl == "c2" and not args.no_bloom
    head = run_hll(ctx, wl, n, args.steps, args.warmup, zipf=args.zipf, groups_n=args.groups,
                   batch_ops=args.batch_ops, bloom_keys=args.bloom_keys if bloom_on else 0)
    result = {
        "metric": "HLL adds/s + Bloom lookups/s (node), % HBM roofline, 1/2/4/8 MI355X",
        "value": head.pop("value"),
        "unit": head.pop("unit"),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head.pop("ms_per_step"),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (splitmix64 %s stream generated on device, untimed)" % wl.upper(),
    }
    for k in ("n_gpus", "steps", "warmup"):
        head.pop(k)
    result.update(head)
    result["rccl_nranks"] = rccl_nranks
    if bloom_on:  # every rank: the node-level Bloom is collective
        bn = args.bloom_keys
        result["bloom"] = bloom_bench(engine, bn, bn, reps=2, rank=rank, world=world,
                                      with_replies=not args.no_bloom_replies)
        tr = pmc_traffic("bloom_insert_supertile", {"workload": wl, "keys": n, "zipf": args.zipf, "bloom_keys": bn}) \
            if world == 1 else None
        if tr:
            ir = result["bloom"]["insert_roofline"]
            ir["traffic"] = tr["bytes"]
            ir["traffic_source"] = tr["source"]
            ir["traffic_GBps"] = tr["bytes"] * ir["achieved"] / ir["algorithmic_bytes"]  # traffic / insert time
    if wl == "c2" and not args.no_extra:
        # the other per-GPU BASELINE configs, each with its own timing and
        # roofline: C4 (configs[3] per GPU: 1B variable-length keys), C5
        # (configs[4] per GPU: 1M sketches, 500M pairs) uniform and Zipf(1.1)
        for key, w2, n2, z in (("c4", "c4", 1_000_000_000, 0.0), ("c5", "c5", 500_000_000, 0.0),
                               ("c5_zipf", "c5", 500_000_000, 1.1)):
            t0 = time.perf_counter()
            result[key] = run_hll(ctx, w2, n2, args.extra_steps, args.extra_warmup, zipf=z, groups_n=args.groups,
                                  batch_ops=args.batch_ops)
            log("%s: %.3f ms/step (%.1f s)" % (key, result[key]["ms_per_step"], time.perf_counter() - t0))
    if rank == 0 and world == 1 and wl == "c2" and not args.no_cpu:
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        result["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.cpu_passes, thr)
        if not args.no_bloom:
            result["cpu_baseline"]["bloom"] = bloom_cpu_baseline(400_000_000, 1 << 24, 1 << 27, thr)
        kd = devmem.gen_keys16(engine, SEED_C2, 0, args.cpu_sample)  # the same C2 stream, copied to host
        host_keys = kd.to_numpy()
        kd.free()
        result["pcie_inclusive"] = pcie_inclusive(client, host_keys)
        del host_keys
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    client.shutdown()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
