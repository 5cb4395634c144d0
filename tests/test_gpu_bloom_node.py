"""The node-level Bloom path that bench.py times (BASELINE configs[2],
north_star "Bloom lookups/s (node)"): inserts sharded over the ranks, partial
bit strings merged by rsk_bloom_allreduce_or, queries sharded over the
replicated filter (RedissonBloomFilter.java:80-168).  On one GPU
it runs with a 1-rank communicator -- exactly the bench's N = 1 path -- and
its bit string must equal the reply-less single-GPU insert and the oracle.
A 2-shard node is emulated on one GPU by inserting each half into its own
filter and OR-merging them, which must again give the single insert."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_C3 = 0x5EED0003


def _bits(L, _lib, b, size):
    out = np.zeros((size + 7) // 8, np.uint8)
    n = ctypes.c_size_t()
    _lib.check(L.rsk_bloom_export_bits(b, out.ctypes.data, out.size, ctypes.byref(n)))
    return out


def test_bench_node_path_equals_single_insert(engine, orc):
    import bench
    from redisson_amd import _lib, devmem, shard

    L = _lib.load()
    n = 3_000_000
    shard.init_comm_single(engine)
    try:
        res = bench.bloom_bench(engine, n, n, reps=1, rank=0, world=1, with_replies=False, keep_bits=True)
    finally:
        _lib.check(L.rsk_comm_destroy(engine.ctx))
    size = ctypes.c_int64()
    k = ctypes.c_int32()
    _lib.check(L.rsk_bloom_params(n, 0.01, _lib.RSK_BLOOM_EXTENDED, ctypes.byref(size), ctypes.byref(k)))
    keys = devmem.gen_keys16(engine, SEED_C3, 0, n)
    b = ctypes.c_void_p()
    _lib.check(L.rsk_bloom_create(engine.ctx, size.value, k.value, ctypes.byref(b)))
    try:
        ks = keys.keys_fixed(n, 16).as_struct()
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
        single = _bits(L, _lib, b, size.value)
    finally:
        L.rsk_bloom_destroy(b)
        keys.free()
    assert np.array_equal(res["bits"], single)
    ref = np.zeros_like(single)
    orc.bloom_add_batch(ref, size.value, k.value, orc.gen_keys16(SEED_C3, 0, n), None, 16, n, want=False)
    assert np.array_equal(single, ref)
    # every inserted query is found; the fresh half stays near the 1 % FPP
    assert res["contains_true"] >= n // 2
    assert res["contains_true"] - n // 2 < 0.03 * (n - n // 2)


def test_two_shard_node_emulated_on_one_gpu(engine, orc):
    """Rank r of a 2-GPU node inserts ShardPlan(n, 2).range(r); OR-merging the
    two partial filters (what rsk_bloom_allreduce_or computes on each rank)
    must give the single-GPU insert of all n keys."""
    from redisson_amd import _lib, devmem, shard

    L = _lib.load()
    n, world = 1_000_003, 2
    size = ctypes.c_int64()
    k = ctypes.c_int32()
    _lib.check(L.rsk_bloom_params(n, 0.01, _lib.RSK_BLOOM_EXTENDED, ctypes.byref(size), ctypes.byref(k)))
    parts = []
    for r in range(world):
        lo, hi = shard.ShardPlan(n, world).range(r)
        keys = devmem.gen_keys16(engine, SEED_C3, lo, hi - lo)
        b = ctypes.c_void_p()
        _lib.check(L.rsk_bloom_create(engine.ctx, size.value, k.value, ctypes.byref(b)))
        ks = keys.keys_fixed(hi - lo, 16).as_struct()
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
        parts.append(b)
        keys.free()
    try:
        other = _bits(L, _lib, parts[1], size.value)
        _lib.check(L.rsk_bloom_or_bits(parts[0], other.ctypes.data, other.size, _lib.RSK_MEM_HOST))
        merged = _bits(L, _lib, parts[0], size.value)
    finally:
        for b in parts:
            L.rsk_bloom_destroy(b)
    ref = np.zeros_like(merged)
    orc.bloom_add_batch(ref, size.value, k.value, orc.gen_keys16(SEED_C3, 0, n), None, 16, n, want=False)
    assert np.array_equal(merged, ref)
