"""RCCL merge layer on one GPU (a 1-rank communicator): the all-reduce paths
run through RCCL and leave single-rank sketches unchanged.  N > 1 exchange
plans are covered bit-exactly on CPU by tests/test_shard_gloo.py."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_one_rank_communicator(engine, orc):
    from redisson_amd import KeyBatch, _lib

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    try:
        h = ctypes.c_void_p()
        _lib.check(L.rsk_hll_create(engine.ctx, 3, ctypes.byref(h)))
        keys = orc.gen_keys16(0x5EED0002, 0, 50000)
        ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
        _lib.check(L.rsk_hll_add(h, 1, ctypes.byref(ks), None))
        ref = np.zeros(16384, np.uint8)
        orc.hll_add(ref, keys, None, 16, 50000)
        _lib.check(L.rsk_hll_allreduce(h, 1))
        _lib.check(L.rsk_hll_allreduce_pool(h))
        first, count = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(L.rsk_hll_reducescatter_pool(h, ctypes.byref(first), ctypes.byref(count)))
        assert (first.value, count.value) == (0, 3)  # one rank owns the whole pool
        fetch = np.array([2, 1, 1, 0], np.uint64)  # all owned: only the count exchange runs
        _lib.check(L.rsk_hll_fetch_rows(h, fetch.ctypes.data, fetch.size))
        _lib.check(L.rsk_hll_fetch_rows(h, None, 0))
        with pytest.raises(_lib.IllegalArgumentException):  # id beyond the pool
            bad = np.array([3], np.uint64)
            _lib.check(L.rsk_hll_fetch_rows(h, bad.ctypes.data, 1))
        out = np.zeros(16384, np.uint8)
        _lib.check(L.rsk_hll_get_registers(h, 1, out.ctypes.data, _lib.RSK_MEM_HOST))
        assert np.array_equal(out, ref)
        cnt = np.zeros(1, np.uint64)
        ids = np.array([1], np.uint64)
        _lib.check(L.rsk_hll_count(h, ids.ctypes.data, 1, cnt.ctypes.data))
        assert int(cnt[0]) == orc.hll_count_dense(ref)
        b = ctypes.c_void_p()
        _lib.check(L.rsk_bloom_create(engine.ctx, 100003, 5, ctypes.byref(b)))
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
        _lib.check(L.rsk_bloom_allreduce_or(b))
        bits = np.zeros((100003 + 7) // 8, np.uint8)
        n = ctypes.c_size_t()
        _lib.check(L.rsk_bloom_export_bits(b, bits.ctypes.data, bits.size, ctypes.byref(n)))
        rb = np.zeros_like(bits)
        orc.bloom_add_batch(rb, 100003, 5, keys, None, 16, 50000, want=False)
        assert np.array_equal(bits, rb)
    finally:
        _lib.check(L.rsk_comm_destroy(engine.ctx))


def test_allreduce_without_comm_is_an_error(engine):
    from redisson_amd import IllegalArgumentException, _lib

    L = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(L.rsk_hll_create(engine.ctx, 1, ctypes.byref(h)))
    with pytest.raises(IllegalArgumentException):
        _lib.check(L.rsk_hll_allreduce(h, 0))


def test_device_memory_roundtrip(engine):
    from redisson_amd import devmem

    a = np.arange(100000, dtype=np.uint64)
    b = devmem.DeviceBuffer.from_numpy(engine, a)
    assert np.array_equal(b.to_numpy(np.uint64), a)
    b.zero()
    assert not b.to_numpy().any()
    b.free()
