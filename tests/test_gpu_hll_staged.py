"""The LDS-staged blob+offsets PFADD path (C4) against the CPU oracle: short
keys of every step count, long keys and empty keys inside staged tiles,
tiles larger than the stage, and blobs that start at every misalignment."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from redisson_amd import _lib

    return _lib.load()


def _add_regs(L, engine, kb):
    from redisson_amd import _lib

    h = ctypes.c_void_p()
    _lib.check(L.rsk_hll_create(engine.ctx, 1, ctypes.byref(h)))
    ch = ctypes.c_uint8()
    ks = kb.as_struct()
    _lib.check(L.rsk_hll_add(h, 0, ctypes.byref(ks), ctypes.byref(ch)))
    out = np.zeros(16384, np.uint8)
    _lib.check(L.rsk_hll_get_registers(h, 0, out.ctypes.data, _lib.RSK_MEM_HOST))
    L.rsk_hll_destroy(h)
    return out


def _batch(seed, n, long_keys=400, wide_run=600):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 48, n)
    lens[rng.integers(0, n, long_keys)] = rng.integers(129, 400, long_keys)  # step class 16 (>= 128 B)
    lens[::997] = 0  # empty keys
    lens[n // 2: n // 2 + wide_run] = 200  # tiles whose bytes exceed the 32 KiB stage
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    blob = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    return blob, offs


def test_staged_mixed_lengths_every_misalignment(L, engine, orc):
    from redisson_amd import KeyBatch, _lib, devmem

    n = 120_000
    blob, offs = _batch(11, n)
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, blob, offs)
    ob = devmem.DeviceBuffer.from_numpy(engine, offs)
    for pad in range(16):
        buf = devmem.DeviceBuffer.from_numpy(engine, np.concatenate([np.zeros(pad, np.uint8), blob]))
        got = _add_regs(L, engine, KeyBatch(buf.ptr + pad, ob.ptr, n, 0, _lib.RSK_MEM_DEVICE, (buf, ob)))
        assert np.array_equal(got, ref), pad
        buf.free()
    # a sub-range whose offsets do not start at 0, and the host-staged copy
    buf = devmem.DeviceBuffer.from_numpy(engine, blob)
    sub = KeyBatch(buf.ptr, ob.ptr, n, 0, _lib.RSK_MEM_DEVICE, (buf, ob)).slice(12345, 100_001)
    o2 = offs[12345:100_002]
    ref2 = np.zeros(16384, np.uint8)
    orc.hll_add(ref2, np.ascontiguousarray(blob[int(o2[0]):int(o2[-1])]), o2 - o2[0])
    assert np.array_equal(_add_regs(L, engine, sub), ref2)
    assert np.array_equal(_add_regs(L, engine, KeyBatch.from_numpy(blob, offs)), ref)
    buf.free()
    ob.free()


@pytest.mark.parametrize("ln", [0, 1, 8, 9, 63, 64])
def test_staged_one_length_per_batch(L, engine, orc, ln):
    """Degenerate tiles: every key in one step class (or every key empty)."""
    from redisson_amd import KeyBatch

    n = 5000
    rng = np.random.default_rng(ln)
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(ln)
    blob = rng.integers(0, 256, n * ln, dtype=np.uint8) if ln else np.zeros(1, np.uint8)
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, blob, offs)
    assert np.array_equal(_add_regs(L, engine, KeyBatch.from_numpy(blob, offs)), ref)
