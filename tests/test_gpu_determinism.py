"""Determinism ("race detection"): the same keys give
identical registers, pools and bit strings whatever their order, however they
are split into calls (so whatever grid each launch gets: a batch below one tile
runs on one workgroup, a large one on the persistent grid) and whether they
come from host or device memory.  MAX and OR are order-independent, so any
difference would be a race (a lost LDS or HBM update)."""
import ctypes

import numpy as np
import pytest

from test_gpu_bloom import _bits, _filter
from test_gpu_hll import _add, _pool, _pool_regs, _regs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from redisson_amd import _lib

    return _lib.load()


def _splits(rng, n, parts):
    cuts = np.sort(rng.choice(np.arange(1, n), parts - 1, replace=False))
    cuts[:3] = [1, 2, 700]  # one-key and sub-tile batches too
    cuts = np.unique(cuts)
    return [0] + cuts.tolist() + [n]


def test_hll_order_and_split_independent(L, engine, orc):
    """5M 16-byte keys: one call; shuffled; in 13 uneven calls (1 key, 1 key,
    698 keys, ...), host-staged; device-resident: all the same registers, equal
    to the oracle.  The same for 300k variable-length keys (the staged kernel's
    class-sorted tiles)."""
    from redisson_amd import KeyBatch, devmem

    rng = np.random.default_rng(11)
    n = 5_000_000
    keys = orc.gen_keys16(0x5EED0002, 0, n).reshape(n, 16)
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, keys.reshape(-1), None, 16, n)
    shuffled = keys[rng.permutation(n)]
    got = []
    for arr, parts in ((keys, 1), (shuffled, 1), (shuffled, 13)):
        h = _pool(L, engine)
        cuts = [0, n] if parts == 1 else _splits(rng, n, parts)
        for a, b in zip(cuts[:-1], cuts[1:]):
            _add(L, h, KeyBatch.from_numpy(np.ascontiguousarray(arr[a:b])))
        got.append(_regs(L, h))
        L.rsk_hll_destroy(h)
    dev = devmem.gen_keys16(engine, 0x5EED0002, 0, n)  # the same stream, device-resident
    h = _pool(L, engine)
    _add(L, h, dev.keys_fixed(n, 16))
    got.append(_regs(L, h))
    L.rsk_hll_destroy(h)
    dev.free()
    for g in got:
        assert np.array_equal(g, ref)
    vk = [rng.integers(0, 256, int(rng.integers(0, 120)), dtype=np.uint8).tobytes() for _ in range(300_000)]
    blob, offs = orc.pack_keys(vk)
    vref = np.zeros(16384, np.uint8)
    orc.hll_add(vref, blob, offs)
    order = rng.permutation(len(vk))
    for perm in (np.arange(len(vk)), order):
        h = _pool(L, engine)
        sub = [vk[i] for i in perm]
        for a, b in zip([0, 5, 70_000], [5, 70_000, len(sub)]):
            _add(L, h, KeyBatch.from_bytes_list(sub[a:b]))
        assert np.array_equal(_regs(L, h), vref)
        L.rsk_hll_destroy(h)


def test_grouped_order_independent(L, engine, orc, route):
    """3M (sketch, key) pairs over 20,000 sketches: in order and shuffled, through
    the partitioned path and the direct one: identical pools."""
    from redisson_amd import KeyBatch, _lib, devmem

    G, n = 20_000, 3_000_000
    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
    groups, keys = g.to_numpy(np.uint32), k.to_numpy().reshape(n, 16)
    g.free()
    k.free()
    perm = np.random.default_rng(5).permutation(n)
    pools = []
    for mode, p in (("1", None), ("1", perm), ("0", perm)):
        route(gpart=1 if mode == "1" else -1)
        gg = groups if p is None else np.ascontiguousarray(groups[p])
        kk = keys if p is None else np.ascontiguousarray(keys[p])
        h = _pool(L, engine, G)
        ks = KeyBatch.from_numpy(kk).as_struct()
        _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), gg.ctypes.data))
        pools.append(_pool_regs(L, engine, h, G))
        L.rsk_hll_destroy(h)
    assert np.array_equal(pools[0], pools[1]) and np.array_equal(pools[0], pools[2])


def test_bloom_order_and_split_independent(L, engine, orc):
    """3M C3 keys into the C3-shaped filter of 2^31 bits (two-level append
    partition): one call, shuffled, and 9 uneven calls (direct-atomic batches
    below 2^22 probes among them) give the same bit string as the oracle."""
    from redisson_amd import KeyBatch, _lib

    rng = np.random.default_rng(3)
    size, k, n = 2_147_483_647, 7, 3_000_000
    keys = orc.gen_keys16(0x5EED0003, 0, n).reshape(n, 16)
    ref = np.zeros((size + 7) // 8, np.uint8)
    orc.bloom_add_batch(ref, size, k, keys.reshape(-1), None, 16, n, want=False)
    shuffled = keys[rng.permutation(n)]
    for arr, parts in ((keys, 1), (shuffled, 1), (shuffled, 9)):
        b = _filter(L, engine, size, k)
        cuts = [0, n] if parts == 1 else _splits(rng, n, parts)
        for a, e in zip(cuts[:-1], cuts[1:]):
            ks = KeyBatch.from_numpy(np.ascontiguousarray(arr[a:e])).as_struct()
            _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
        assert np.array_equal(_bits(L, b, size), ref)
        L.rsk_bloom_destroy(b)
