"""Bloom parity: gfx950 kernels against the CPU oracle (bit-exact bit strings,
identical add/contains replies), through the C ABI."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


@pytest.fixture(scope="module")
def L():
    from redisson_amd import _lib

    return _lib.load()


def _filter(L, engine, size, k):
    from redisson_amd import _lib

    b = ctypes.c_void_p()
    _lib.check(L.rsk_bloom_create(engine.ctx, size, k, ctypes.byref(b)))
    return b


def _bits(L, b, size):
    from redisson_amd import _lib

    out = np.zeros((size + 7) // 8, np.uint8)
    n = ctypes.c_size_t()
    _lib.check(L.rsk_bloom_export_bits(b, out.ctypes.data, out.size, ctypes.byref(n)))
    assert n.value == out.size
    return out


def _add(L, b, kb, replies=True):
    from redisson_amd import _lib

    out = np.zeros(max(1, kb.n), np.uint8)
    ks = kb.as_struct()
    _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), out.ctypes.data if replies else None))
    return out[: kb.n]


def _contains(L, b, kb):
    from redisson_amd import _lib

    out = np.zeros(max(1, kb.n), np.uint8)
    ks = kb.as_struct()
    _lib.check(L.rsk_bloom_contains(b, ctypes.byref(ks), out.ctypes.data))
    return out[: kb.n]


def test_golden_c3_insert(L, engine, orc):
    from redisson_amd import KeyBatch

    g = GOLDEN["bloom_c3_10000"]
    keys = orc.gen_keys16(0x5EED0003, 0, 10000)
    b = _filter(L, engine, g["size"], g["k"])
    added = _add(L, b, KeyBatch.from_numpy(keys.reshape(-1, 16)))
    bits = _bits(L, b, g["size"])
    assert hashlib.sha256(bits.tobytes()).hexdigest() == g["bits_sha256"]
    assert int(added.sum()) == g["added_true"]
    ref_bits = np.zeros_like(bits)
    ref_added = orc.bloom_add_batch(ref_bits, g["size"], g["k"], keys, None, 16, 10000)
    assert np.array_equal(added, ref_added)
    c = ctypes.c_int32()
    assert L.rsk_bloom_count(b, ctypes.byref(c)) == 0 and c.value == g["count"]


@pytest.mark.parametrize("size,k", [(729, 5), (95851, 7), (1000003, 33), (64, 3), (1, 2), (4014142460, 5)])
def test_add_contains_varlen_parity(L, engine, orc, size, k):
    from redisson_amd import KeyBatch

    rng = np.random.default_rng(size % 1000 + k)
    keys = [rng.integers(0, 256, int(rng.integers(0, 150)), dtype=np.uint8).tobytes() for _ in range(3000)]
    keys += keys[:500] + [b"", b""]  # duplicates inside one batch
    b = _filter(L, engine, size, k)
    kb = KeyBatch.from_bytes_list(keys)
    added = _add(L, b, kb)
    blob, offs = orc.pack_keys(keys)
    ref_bits = np.zeros((size + 7) // 8, np.uint8)
    ref_added = orc.bloom_add_batch(ref_bits, size, k, blob, offs)
    assert np.array_equal(added, ref_added)
    if size < (1 << 28):
        assert np.array_equal(_bits(L, b, size), ref_bits)
    q = keys[:1000] + [rng.integers(0, 256, 20, dtype=np.uint8).tobytes() for _ in range(1000)]
    qb, qo = orc.pack_keys(q)
    if size < (1 << 28):
        want = orc.bloom_contains_batch(ref_bits, size, k, qb, qo)
    else:
        want = None
    got = _contains(L, b, KeyBatch.from_bytes_list(q))
    assert got[:1000].all() or k == 1
    if want is not None:
        assert np.array_equal(got, want)


def test_c3_stream_device_resident(L, engine, orc):
    from redisson_amd import _lib, devmem

    n_ins, n_q = 2_000_000, 2_000_000
    size = orc.bloom_optimal_bits(n_ins, 0.01)
    k = orc.bloom_optimal_k(n_ins, size)
    ins = devmem.gen_keys16(engine, 0x5EED0003, 0, n_ins)
    qs = devmem.gen_queries16(engine, 0x5EED0004, 0x5EED0003, n_ins, 0, n_q)
    b = _filter(L, engine, size, k)
    ks = ins.keys_fixed(n_ins, 16).as_struct()
    _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
    out = devmem.DeviceBuffer(engine, n_q)
    qk = qs.keys_fixed(n_q, 16).as_struct()
    _lib.check(L.rsk_bloom_contains(b, ctypes.byref(qk), out.ptr))
    engine.sync()
    ref_bits = np.zeros((size + 7) // 8, np.uint8)
    orc.bloom_add_batch(ref_bits, size, k, ins.to_numpy(), None, 16, n_ins, want=False)
    assert np.array_equal(_bits(L, b, size), ref_bits)
    qn = qs.to_numpy()
    assert np.array_equal(qn, orc.gen_queries16(0x5EED0004, 0x5EED0003, n_ins, 0, n_q))
    want = orc.bloom_contains_batch(ref_bits, size, k, qn, None, 16, n_q)
    got = out.to_numpy()
    assert np.array_equal(got, want)
    # every inserted key is found; the fresh half shows a ~1% false-positive rate
    bc = ctypes.c_uint64()
    assert L.rsk_bloom_bitcount(b, ctypes.byref(bc)) == 0 and bc.value == orc.bitcount(ref_bits)


@pytest.mark.parametrize("size,k,n", [(1, 2, 5000), (729, 5, 20000), (95851, 7, 50000), (1000003, 33, 20000),
                                      (19170117, 7, 300000), (157298745, 7, 400000), (157298745, 3, 700000)])
def test_partitioned_add_parity(L, engine, orc, route, size, k, n):
    """Slice-partitioned add (forced on) gives the oracle's bit string: one partition
    level (<= 256 slices of 2^19 bits) and two levels (157M bits = 301 slices)."""
    from redisson_amd import KeyBatch

    route(bloom_part=1, bloom_stream=-1)
    keys = orc.gen_keys16(0x5EED0003, 0, n)
    b = _filter(L, engine, size, k)
    _add(L, b, KeyBatch.from_numpy(keys.reshape(-1, 16)), replies=False)
    ref = np.zeros((size + 7) // 8, np.uint8)
    orc.bloom_add_batch(ref, size, k, keys, None, 16, n, want=False)
    assert np.array_equal(_bits(L, b, size), ref)
    # variable-length keys (blob + offsets) and duplicates through the same path
    rng = np.random.default_rng(k)
    vk = [rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes() for _ in range(4000)]
    vk += vk[:1000] + [b""]
    _add(L, b, KeyBatch.from_bytes_list(vk), replies=False)
    blob, offs = orc.pack_keys(vk)
    orc.bloom_add_batch(ref, size, k, blob, offs, want=False)
    assert np.array_equal(_bits(L, b, size), ref)


ST_CASES = [(1, 2, 5000), (729, 5, 20000), (95851, 7, 50000), (1000003, 1, 50000), (19170117, 7, 300000),
            (157298745, 7, 400000), (157298745, 9, 200000), (157298745, 16, 150000), (4014142460, 8, 600000)]


ST_KNOBS = ["bloom_stream=1", "bloom_stream=1,bloom_chunk=300000", "bloom_stream=1,sa_tiny=1",
            "bloom_stream=1,sa_parts=1", "bloom_stream=1,sa_parts=13"]


@pytest.mark.parametrize("size,k,n", ST_CASES)
@pytest.mark.parametrize("knobs", ST_KNOBS)
def test_slice_routed_add_parity(L, engine, orc, route, size, k, n, knobs):
    """The slice-routed insert (rsk_bloom_st.hip), forced on, gives the oracle's
    bit string: one level (<= 256 slices: st1 + apply) and two (301, 7,657 and
    7,657 slices through the append pipeline sa1/sa2/apply), k in {1, 2, 5, 7,
    8} (2 or 4 keys per lane) and {9, 16} (1 key per lane); many chunks;
    sub-regions too small (overflow into the exact-offset fallback); sa2 with
    one part per coarse bin (every workgroup walks all sub-regions) and with 13
    (parts without any sub-region when the batch has few super-tiles)."""
    from redisson_amd import KeyBatch

    route(knobs)
    keys = orc.gen_keys16(0x5EED0003, 0, n)
    b = _filter(L, engine, size, k)
    _add(L, b, KeyBatch.from_numpy(keys.reshape(-1, 16)), replies=False)
    ref = np.zeros((size + 7) // 8, np.uint8)
    orc.bloom_add_batch(ref, size, k, keys, None, 16, n, want=False)
    assert np.array_equal(_bits(L, b, size), ref)
    # variable-length keys (blob + offsets, the generic hashing branch) and duplicates
    rng = np.random.default_rng(k + n)
    vk = [rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes() for _ in range(4000)]
    vk += vk[:1000] + [b""]
    _add(L, b, KeyBatch.from_bytes_list(vk), replies=False)
    blob, offs = orc.pack_keys(vk)
    orc.bloom_add_batch(ref, size, k, blob, offs, want=False)
    assert np.array_equal(_bits(L, b, size), ref)
    L.rsk_bloom_destroy(b)


@pytest.mark.parametrize("knobs", ST_KNOBS)
def test_slice_routed_skewed_keys(L, engine, orc, route, knobs):
    """One key repeated 300,000 times plus a few distinct ones: every probe of
    the repeated key lands in the same k slices (one long segment per
    super-tile and bin), so st2 tiles and apply segments are full-length runs."""
    from redisson_amd import KeyBatch

    route(knobs)
    size, k = 157298745, 7
    base = orc.gen_keys16(0x5EED0003, 0, 1000).reshape(-1, 16)
    keys = np.concatenate([np.repeat(base[:1], 300000, axis=0), base[1:]]).reshape(-1)
    b = _filter(L, engine, size, k)
    _add(L, b, KeyBatch.from_numpy(keys.reshape(-1, 16)), replies=False)
    ref = np.zeros((size + 7) // 8, np.uint8)
    orc.bloom_add_batch(ref, size, k, keys, None, 16, keys.size // 16, want=False)
    assert np.array_equal(_bits(L, b, size), ref)
    L.rsk_bloom_destroy(b)


def test_slice_routed_matches_direct_c3_size(L, engine, route):
    """At the C3 filter size (9,585,058,377 bits, 18,283 slices: 143 coarse bins
    x 128 slices) the super-tile insert and the direct atomicOr kernel set
    identical bits."""
    from redisson_amd import _lib, devmem

    size, k, n = 9585058377, 7, 3_000_000
    ins = devmem.gen_keys16(engine, 0x5EED0003, 0, n)
    ks = ins.keys_fixed(n, 16).as_struct()
    filters = {}
    for mode in ("1", "0"):
        route(bloom_stream=1 if mode == "1" else -1, bloom_part=-1)
        f = _filter(L, engine, size, k)
        _lib.check(L.rsk_bloom_add(f, ctypes.byref(ks), None))
        filters[mode] = f
    engine.sync()
    counts = {}
    for mode, f in filters.items():
        bc = ctypes.c_uint64()
        _lib.check(L.rsk_bloom_bitcount(f, ctypes.byref(bc)))
        counts[mode] = bc.value
    assert counts["1"] == counts["0"] > 0.99 * n * k
    nbytes = (size + 7) // 8
    _lib.check(L.rsk_bloom_or_bits(filters["1"], L.rsk_bloom_device_bits(filters["0"]), nbytes, _lib.RSK_MEM_DEVICE))
    bc = ctypes.c_uint64()
    _lib.check(L.rsk_bloom_bitcount(filters["1"], ctypes.byref(bc)))
    assert bc.value == counts["0"]
    for f in filters.values():
        L.rsk_bloom_destroy(f)
    ins.free()


def test_partitioned_add_matches_direct_c3_size(L, engine, route):
    """At the C3 filter size (9,585,058,377 bits, 18,283 slices, two levels) the
    exact-offset partitioned add (the k > 16 path and the super-tile fallback)
    and the direct atomicOr kernel set identical bits."""
    from redisson_amd import _lib, devmem

    size, k, n = 9585058377, 7, 3_000_000
    ins = devmem.gen_keys16(engine, 0x5EED0003, 0, n)
    ks = ins.keys_fixed(n, 16).as_struct()
    filters = {}
    for mode in ("1", "0"):
        route(bloom_stream=-1, bloom_part=1 if mode == "1" else -1)
        f = _filter(L, engine, size, k)
        _lib.check(L.rsk_bloom_add(f, ctypes.byref(ks), None))
        filters[mode] = f
    engine.sync()
    counts = {}
    for mode, f in filters.items():
        bc = ctypes.c_uint64()
        _lib.check(L.rsk_bloom_bitcount(f, ctypes.byref(bc)))
        counts[mode] = bc.value
    assert counts["1"] == counts["0"] > 0.99 * n * k
    # partitioned |= direct leaves the count unchanged  =>  the bit strings are equal
    nbytes = (size + 7) // 8
    _lib.check(L.rsk_bloom_or_bits(filters["1"], L.rsk_bloom_device_bits(filters["0"]), nbytes, _lib.RSK_MEM_DEVICE))
    bc = ctypes.c_uint64()
    _lib.check(L.rsk_bloom_bitcount(filters["1"], ctypes.byref(bc)))
    assert bc.value == counts["0"]
    for f in filters.values():
        L.rsk_bloom_destroy(f)
    ins.free()


def test_or_bits_merge(L, engine, orc):
    from redisson_amd import KeyBatch, _lib

    size, k = 100003, 5
    keys = orc.gen_keys16(0x5EED0003, 0, 20000).reshape(-1, 16)
    a = _filter(L, engine, size, k)
    b = _filter(L, engine, size, k)
    full = _filter(L, engine, size, k)
    _add(L, a, KeyBatch.from_numpy(keys[:10000]), replies=False)
    _add(L, b, KeyBatch.from_numpy(keys[10000:]), replies=False)
    _add(L, full, KeyBatch.from_numpy(keys), replies=False)
    bb = _bits(L, b, size)
    _lib.check(L.rsk_bloom_or_bits(a, bb.ctypes.data, bb.size, _lib.RSK_MEM_HOST))
    assert np.array_equal(_bits(L, a, size), _bits(L, full, size))


def test_c3_full_size_bit_exact(L, engine, orc):
    """BASELINE configs[2] at full size: 1B inserts at 1% FPP (EXTENDED,
    9,585,058,377 bits, k=7) through the slice-partitioned insert, then 1B
    contains(); the bit string and every reply equal the oracle's (OpenMP
    restatement of the same streams)."""
    import os

    from redisson_amd import _lib, devmem

    n = 1_000_000_000
    size, k = 9585058377, 7
    threads = max(1, min(16, os.cpu_count() or 1))
    ins = devmem.gen_keys16(engine, 0x5EED0003, 0, n)
    b = _filter(L, engine, size, k)
    ks = ins.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
    ins.free()
    qs = devmem.gen_queries16(engine, 0x5EED0004, 0x5EED0003, n, 0, n)
    out = devmem.DeviceBuffer(engine, n)
    qk = qs.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_bloom_contains(b, ctypes.byref(qk), out.ptr))
    qs.free()
    got_bits = _bits(L, b, size)
    got = out.to_numpy()
    out.free()
    L.rsk_bloom_destroy(b)
    ref_bits = np.zeros((size + 7) // 8, np.uint8)
    orc.bloom_add_gen16_mt(ref_bits, size, k, 0x5EED0003, 0, n, threads)
    assert np.array_equal(got_bits, ref_bits)
    del got_bits
    want = np.zeros(n, np.uint8)
    trues = orc.bloom_contains_gen_queries_mt(ref_bits, size, k, 0x5EED0004, 0x5EED0003, n, 0, n, want, threads)
    assert np.array_equal(got, want)
    assert 0.50 < trues / n < 0.52  # half members + ~1% false positives on the fresh half


@pytest.mark.parametrize("copy", [0, -1])
def test_large_filter_bits_round_trip(L, engine, route, copy):
    """A filter of 2^30 + 12345 bits (128 MiB, not a whole number of 16 MiB
    pieces): SET of a random bit string (rsk_bloom_import_bits, through the
    pinned stages) then GET (rsk_bloom_export_bits, through the D2H ring on
    the measured SDMA engine -- route io_engine = 0 -- or HIP's copies, -1;
    and straight into a caller-registered buffer) returns the same bytes, and
    BITCOUNT equals the host popcount."""
    from redisson_amd import _lib

    route(io_engine=copy)
    size = (1 << 30) + 12345
    nb = (size + 7) // 8
    rng = np.random.default_rng(33)
    src = rng.integers(0, 256, nb, dtype=np.uint8)
    src[-1] &= 0xFF << (8 - size % 8) & 0xFF  # (bits past size stay clear)
    b = _filter(L, engine, size, 3)
    _lib.check(L.rsk_bloom_import_bits(b, src.ctypes.data, src.size))
    assert np.array_equal(_bits(L, b, size), src)
    bc = ctypes.c_uint64()
    _lib.check(L.rsk_bloom_bitcount(b, ctypes.byref(bc)))
    assert bc.value == int(np.unpackbits(src).sum())
    reg = np.zeros(nb + 4096, np.uint8)
    engine.host_register(reg)
    try:
        n = ctypes.c_size_t()
        _lib.check(L.rsk_bloom_export_bits(b, reg.ctypes.data, reg.size, ctypes.byref(n)))
        assert n.value == nb and np.array_equal(reg[:nb], src)
    finally:
        engine.host_unregister(reg)
    L.rsk_bloom_destroy(b)
