"""Host-resident batches spread over many staging chunks: the double-buffered
pinned stages (par_copy by host threads while the other stage's DMA runs)
must give the same registers / bits / replies as the oracle and as one-chunk
batches.  A 32 MiB stage makes every batch here 3-6 chunks, each copied by
several threads; batches of 64 MiB or more go up on the SDMA engine measured
fastest (route io_engine = 0) or on HIP's copies (-1), both run."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STAGE = 32 << 20
SEED_C2 = 0x5EED0002


@pytest.fixture(scope="module")
def L():
    from redisson_amd import _lib

    return _lib.load()


@pytest.fixture(scope="module")
def small_engine_ctx():
    from redisson_amd import _lib

    e = _lib.Engine(0, staging_bytes=STAGE)
    yield e
    e.close()


@pytest.fixture(params=[0, -1], ids=["engine", "hip"])
def small_engine(request, small_engine_ctx):
    small_engine_ctx.set_route("io_engine", request.param)
    yield small_engine_ctx
    small_engine_ctx.set_route("reset", 0)


def _regs_after_add(L, engine, kb):
    from redisson_amd import _lib

    h = ctypes.c_void_p()
    _lib.check(L.rsk_hll_create(engine.ctx, 1, ctypes.byref(h)))
    ch = ctypes.c_uint8()
    ks = kb.as_struct()
    _lib.check(L.rsk_hll_add(h, 0, ctypes.byref(ks), ctypes.byref(ch)))
    out = np.zeros(16384, np.uint8)
    _lib.check(L.rsk_hll_get_registers(h, 0, out.ctypes.data, _lib.RSK_MEM_HOST))
    L.rsk_hll_destroy(h)
    return out, bool(ch.value)


def test_staged_fixed16_many_chunks(L, small_engine, orc):
    from redisson_amd import KeyBatch

    n = 6_000_000  # 96 MB of keys: 3 chunks of 32 MiB
    keys = orc.gen_keys16(SEED_C2, 0, n)
    ref = np.zeros(16384, np.uint8)
    orc.hll_add_gen16(ref, SEED_C2, 0, n, 8)
    got, changed = _regs_after_add(L, small_engine, KeyBatch.from_numpy(keys.reshape(n, 16)))
    assert changed
    assert np.array_equal(got, ref)


def test_staged_varlen_many_chunks(L, small_engine, orc):
    from redisson_amd import KeyBatch

    rng = np.random.default_rng(7)
    n = 3_000_000
    lens = rng.integers(8, 65, n)
    lens[::1001] = 0
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    blob = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)  # ~109 MB: 4 chunks
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, blob, offs)
    got, _ = _regs_after_add(L, small_engine, KeyBatch.from_numpy(blob, offs))
    assert np.array_equal(got, ref)
    # a sub-range whose offsets do not start at 0
    sub = KeyBatch.from_numpy(blob, offs).slice(777, n - 5)
    o2 = offs[777:n - 4]
    ref2 = np.zeros(16384, np.uint8)
    orc.hll_add(ref2, np.ascontiguousarray(blob[int(o2[0]):int(o2[-1])]), o2 - o2[0])
    got2, _ = _regs_after_add(L, small_engine, sub)
    assert np.array_equal(got2, ref2)


def test_staged_bloom_replies_match_one_chunk(L, small_engine, engine, orc):
    from redisson_amd import KeyBatch, _lib

    n = 4_000_000  # 64 MB of 16-byte keys: 2 chunks; replies in 2 sub-batches
    keys = orc.gen_keys16(0xB100, 0, n).reshape(n, 16)
    fresh = orc.gen_keys16(0xB101, 0, n).reshape(n, 16)
    size, k = 40_000_000, 5
    outs = []
    for eng in (small_engine, engine):
        b = ctypes.c_void_p()
        _lib.check(L.rsk_bloom_create(eng.ctx, size, k, ctypes.byref(b)))
        added = np.zeros(n, np.uint8)
        ks = KeyBatch.from_numpy(keys).as_struct()
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), added.ctypes.data))
        hit = np.zeros(2 * n, np.uint8)
        both = np.concatenate([keys, fresh])
        qs = KeyBatch.from_numpy(both).as_struct()
        _lib.check(L.rsk_bloom_contains(b, ctypes.byref(qs), hit.ctypes.data))
        L.rsk_bloom_destroy(b)
        outs.append((added, hit))
    (a0, h0), (a1, h1) = outs
    assert np.array_equal(a0, a1)
    assert np.array_equal(h0, h1)
    assert h0[:n].all()  # every inserted key is a member
    assert 0 < int(h0[n:].sum()) < n // 10  # fresh keys: false positives only
