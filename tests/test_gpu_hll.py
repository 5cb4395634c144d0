"""HLL parity: the gfx950 kernels against the CPU oracle (bit-exact registers,
exact PFCOUNT results), through the C ABI."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
SEED_C2 = 0x5EED0002
SEED_C4 = 0x5EED0005


@pytest.fixture(scope="module")
def L():
    from redisson_amd import _lib

    return _lib.load()


def _pool(L, engine, n=1):
    from redisson_amd import _lib

    h = ctypes.c_void_p()
    _lib.check(L.rsk_hll_create(engine.ctx, n, ctypes.byref(h)))
    return h


def _regs(L, h, i=0):
    from redisson_amd import _lib

    out = np.zeros(16384, np.uint8)
    _lib.check(L.rsk_hll_get_registers(h, i, out.ctypes.data, _lib.RSK_MEM_HOST))
    return out


def _add(L, h, kb, i=0):
    from redisson_amd import _lib

    ch = ctypes.c_uint8()
    ks = kb.as_struct()
    _lib.check(L.rsk_hll_add(h, i, ctypes.byref(ks), ctypes.byref(ch)))
    return bool(ch.value)


def _count(L, h, ids):
    from redisson_amd import _lib

    ids = np.asarray(ids, np.uint64)
    out = np.zeros(ids.size, np.uint64)
    _lib.check(L.rsk_hll_count(h, ids.ctypes.data, ids.size, out.ctypes.data))
    return out


def test_add16_matches_oracle(L, engine, orc):
    from redisson_amd import KeyBatch

    for n in (1, 7, 100, 1000, 20000, 200000, 1 << 20):
        keys = orc.gen_keys16(SEED_C2, 0, n)
        h = _pool(L, engine)
        assert _add(L, h, KeyBatch.from_numpy(keys.reshape(n, 16)))
        ref = np.zeros(16384, np.uint8)
        orc.hll_add(ref, keys, None, 16, n)
        got = _regs(L, h)
        assert np.array_equal(got, ref), n
        c = int(_count(L, h, [0])[0])
        assert c == orc.hll_count_dense(ref) == orc.hll_count_raw(ref)
        g = GOLDEN["hll"].get("c2_%d" % n)
        if g:
            assert hashlib.sha256(got.tobytes()).hexdigest() == g["registers_sha256"]
            assert c == g["count_dense"]
        L.rsk_hll_destroy(h)


def test_add_device_resident_keys(L, engine, orc):
    from redisson_amd import devmem

    n = 3_000_000
    t = devmem.gen_keys16(engine, SEED_C2, 0, n)
    assert np.array_equal(t.to_numpy(), orc.gen_keys16(SEED_C2, 0, n))
    kb = t.keys_fixed(n, 16)
    h = _pool(L, engine)
    _add(L, h, kb)
    ref = np.zeros(16384, np.uint8)
    orc.hll_add_gen16(ref, SEED_C2, 0, n, 8)
    assert np.array_equal(_regs(L, h), ref)
    # idempotence: re-adding the same keys changes nothing -> PFADD replies 0
    assert not _add(L, h, kb)
    # chunk-order independence: two halves into a fresh sketch
    h2 = _pool(L, engine)
    _add(L, h2, kb.slice(n // 2, n))
    _add(L, h2, kb.slice(0, n // 2))
    assert np.array_equal(_regs(L, h2), ref)
    # misaligned device keys take the generic path and agree
    h3 = _pool(L, engine)
    _add(L, h3, t.keys_fixed(n // 2 - 1, 16, offset=8))
    ref3 = np.zeros(16384, np.uint8)
    raw = orc.gen_keys16(SEED_C2, 0, n // 2)[8:8 + 16 * (n // 2 - 1)]
    orc.hll_add(ref3, raw, None, 16, n // 2 - 1)
    assert np.array_equal(_regs(L, h3), ref3)


@pytest.mark.parametrize("fixed_len", [1, 3, 7, 8, 9, 15, 17, 31, 33, 64, 65, 100])
def test_add_fixed_lengths(L, engine, orc, fixed_len):
    from redisson_amd import KeyBatch

    rng = np.random.default_rng(fixed_len)
    n = 50000
    keys = rng.integers(0, 256, n * fixed_len, dtype=np.uint8)
    h = _pool(L, engine)
    _add(L, h, KeyBatch.from_numpy(keys.reshape(n, fixed_len)))
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, keys, None, fixed_len, n)
    assert np.array_equal(_regs(L, h), ref)


def test_add_variable_length_and_empty(L, engine, orc):
    from redisson_amd import KeyBatch

    rng = np.random.default_rng(7)
    keys = [rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes() for _ in range(30000)]
    keys += [b"", b"", b"x"]
    h = _pool(L, engine)
    _add(L, h, KeyBatch.from_bytes_list(keys))
    blob, offs = orc.pack_keys(keys)
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, blob, offs)
    assert np.array_equal(_regs(L, h), ref)


def test_varlen_c4_stream(L, engine, orc):
    from redisson_amd import devmem

    n = 200000
    blob, offs, tot = devmem.gen_varlen(engine, SEED_C4, 0, n)
    rblob, roffs = orc.gen_varlen(SEED_C4, 0, n)
    assert np.array_equal(offs.to_numpy(np.uint64), roffs)
    assert np.array_equal(blob.to_numpy(count=tot), rblob[: int(roffs[-1])])
    h = _pool(L, engine)
    _add(L, h, blob.keys_var(offs, n))
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, rblob, roffs)
    assert np.array_equal(_regs(L, h), ref)


def test_count_cache_and_union_and_merge(L, engine, orc):
    from redisson_amd import KeyBatch, _lib

    h = _pool(L, engine, 4)
    sets = []
    for i, n in enumerate((10, 5000, 60000, 400000)):
        keys = orc.gen_keys16(SEED_C2 + i, 0, n)
        _add(L, h, KeyBatch.from_numpy(keys.reshape(n, 16)), i)
        ref = np.zeros(16384, np.uint8)
        orc.hll_add(ref, keys, None, 16, n)
        sets.append(ref)
    got = _count(L, h, [0, 1, 2, 3, 3, 0])
    want = [orc.hll_count_dense(r) for r in sets]
    assert list(got) == want + [want[3], want[0]]
    # union (countWith): raw-order estimator on the max registers
    for members in ([0, 1], [1, 2, 3], [3, 3], [0, 1, 2, 3]):
        pools = (ctypes.c_void_p * len(members))(*([h.value] * len(members)))
        ids = (ctypes.c_uint64 * len(members))(*members)
        out = (ctypes.c_uint64 * 1)()
        _lib.check(L.rsk_hll_count_union(pools, ids, len(members), out))
        mx = np.maximum.reduce([sets[m] for m in members])
        assert out[0] == orc.hll_count_raw(mx)
    # merge (PFMERGE 0 <- 1,2): dest included
    pools = (ctypes.c_void_p * 2)(h.value, h.value)
    ids = (ctypes.c_uint64 * 2)(1, 2)
    _lib.check(L.rsk_hll_merge(h, 0, pools, ids, 2))
    mx = np.maximum.reduce([sets[0], sets[1], sets[2]])
    assert np.array_equal(_regs(L, h, 0), mx)
    assert int(_count(L, h, [0])[0]) == orc.hll_count_dense(mx)


def test_count_inexact_fallback(L, engine, orc):
    """Registers spanning > 53 bits force the ordered (dense) summation."""
    from redisson_amd import _lib

    rng = np.random.default_rng(3)
    for trial in range(4):
        regs = rng.integers(1, 4, 16384).astype(np.uint8)  # no zeros, small ranks
        regs[rng.integers(0, 16384, 40)] = rng.integers(44, 51, 40).astype(np.uint8)
        h = _pool(L, engine)
        _lib.check(L.rsk_hll_merge_raw(h, 0, regs.ctypes.data, _lib.RSK_MEM_HOST))
        assert int(_count(L, h, [0])[0]) == orc.hll_count_dense(regs)
        pools = (ctypes.c_void_p * 1)(h.value)
        ids = (ctypes.c_uint64 * 1)(0)
        out = (ctypes.c_uint64 * 1)()
        _lib.check(L.rsk_hll_count_union(pools, ids, 1, out))
        assert out[0] == orc.hll_count_raw(regs)


def test_export_import_redis_strings(L, engine, orc):
    from redisson_amd import KeyBatch, _lib

    keys = orc.gen_keys16(SEED_C2, 0, 2000)
    h = _pool(L, engine, 2)
    _add(L, h, KeyBatch.from_numpy(keys.reshape(-1, 16)), 0)
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, keys, None, 16, 2000)
    buf = (ctypes.c_uint8 * 12304)()
    n = ctypes.c_size_t()
    _lib.check(L.rsk_hll_export_redis(h, 0, buf, 12304, ctypes.byref(n)))
    s = bytes(buf[: n.value])
    assert n.value == 12304 and s[:5] == b"HYLL\x00"
    rc, raw, enc = orc.hll_decode(s)
    assert rc == 0 and enc == 0 and np.array_equal(raw, ref)
    assert s[16:] == orc.hll_encode_dense(ref)[16:]
    assert s[15] & 0x80  # cache invalid after PFADD
    # import a sparse string produced by the oracle into slot 1
    sp = orc.hll_encode_sparse(ref)
    b = (ctypes.c_uint8 * len(sp)).from_buffer_copy(sp)
    _lib.check(L.rsk_hll_import_redis(h, 1, b, len(sp)))
    assert np.array_equal(_regs(L, h, 1), ref)
    assert int(_count(L, h, [1])[0]) == orc.hll_count_string(sp)[1]
    bad = (ctypes.c_uint8 * 20).from_buffer_copy(b"HYLL\x00" + b"\0" * 15)
    assert L.rsk_hll_import_redis(h, 1, bad, 20) == _lib.RSK_ERR_WRONGTYPE


def test_add_each_matches_sequential_pfadd(L, engine, orc):
    from redisson_amd import KeyBatch, _lib

    rng = np.random.default_rng(11)
    base = [rng.integers(0, 256, 12, dtype=np.uint8).tobytes() for _ in range(20000)]
    keys = base + base[:5000] + [base[7]] * 3  # duplicates -> later replies 0
    r = orc.RedisModel()
    want = [r.pfadd("k", e) for e in keys]
    h = _pool(L, engine)
    out = np.zeros(len(keys), np.uint8)
    ks = KeyBatch.from_bytes_list(keys).as_struct()
    _lib.check(L.rsk_hll_add_each(h, 0, ctypes.byref(ks), out.ctypes.data))
    assert out.tolist() == want
    rc, raw, _ = orc.hll_decode(r.get("k"))
    assert np.array_equal(_regs(L, h), raw)


def test_grouped_add_matches_oracle(L, engine, orc):
    from redisson_amd import _lib, devmem

    G, n = 1000, 2_000_000
    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
    rg, rk = orc.gen_grouped(0x5EED0006, G, 0, n)
    assert np.array_equal(g.to_numpy(np.uint32), rg) and np.array_equal(k.to_numpy(), rk)
    h = _pool(L, engine, G)
    ks = k.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    ref = np.zeros(G * 16384, np.uint8)
    orc.hll_add_gen_grouped(ref, G, 0x5EED0006, 0, n)
    for gid in list(range(0, G, 37)) + [G - 1]:
        assert np.array_equal(_regs(L, h, gid), ref[gid * 16384:(gid + 1) * 16384]), gid
    ids = np.arange(G, dtype=np.uint64)
    out = np.zeros(G, np.uint64)
    _lib.check(L.rsk_hll_count(h, ids.ctypes.data, G, out.ctypes.data))
    want = [orc.hll_count_dense(ref[i * 16384:(i + 1) * 16384]) for i in range(G)]
    assert out.tolist() == want


def _pool_regs(L, engine, h, G):
    from redisson_amd import _lib

    out = np.zeros(G * 16384, np.uint8)
    _lib.check(L.rsk_memcpy(engine.ctx, out.ctypes.data, L.rsk_hll_device_registers(h), out.nbytes, 1))
    return out


@pytest.mark.parametrize("tm", [0, 1])
@pytest.mark.parametrize("G,n", [(8205, 3_000_000), (1, 50_000), (4096 * 3, 2_000_001), (20, 4_500_003)])
def test_grouped_partitioned_matches_direct_and_oracle(L, engine, orc, route, G, n, tm):
    """Grouped PFADD partitioned by sketch (coarse bins of 4096 sketches, fine
    bins of 16, LDS halves of 8; G not a multiple of any of them) equals the
    direct random-CAS kernel and the oracle over the whole pool; tm=1 takes the
    tile-major first pass (hll_gpart1t)."""
    from redisson_amd import _lib, devmem

    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
    ks = k.keys_fixed(n, 16).as_struct()
    pools = {}
    for mode in ("1", "0"):
        route(gpart=1 if mode == "1" else -1, gpart_tm=tm)
        h = _pool(L, engine, G)
        _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
        pools[mode] = h
    g.free()
    k.free()
    part, direct = (_pool_regs(L, engine, pools[m], G) for m in ("1", "0"))
    assert np.array_equal(part, direct)
    ref = np.zeros(G * 16384, np.uint8)
    orc.hll_add_gen_grouped(ref, G, 0x5EED0006, 0, n)
    assert np.array_equal(part, ref)
    for h in pools.values():
        L.rsk_hll_destroy(h)


@pytest.mark.parametrize("tm", [0, 1, 2])  # 2: tile-major with 16384-record tiles (route gpart_tile)
@pytest.mark.parametrize("G,n,zipf", [(4096 * 10 + 16, 50_000_000, 0.0), (1_000_000, 60_000_000, 0.0),
                                      (200_000, 40_000_000, 1.1)])
def test_grouped_partitioned_leaves_no_holes(L, engine, route, G, n, zipf, tm):
    """The fine-bin pass writes every slot the counts reserve: with its output
    poisoned (0xFF records first: a slot left unwritten would raise a register
    to 63) the partitioned add still equals the direct kernel.  Sizes where a
    bin's segments are a few records per tile (the last, nearly empty coarse
    bin; Zipf's cold bins) and rounds end at the window's tile count."""
    from redisson_amd import _lib, devmem

    if zipf:
        g, k = devmem.gen_grouped_zipf(engine, 0x5EED0007, G, zipf, 0, n)
    else:
        g, k = devmem.gen_grouped(engine, 0x5EED0007, G, 0, n)
    ks = k.keys_fixed(n, 16).as_struct()
    pools = {}
    for mode in ("1", "0"):
        route(gpart=1 if mode == "1" else -1, gpart_tm=min(tm, 1), gpart_tile=int(tm == 2), gpart_poison=1)
        h = _pool(L, engine, G)
        _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
        pools[mode] = h
    g.free()
    k.free()
    part, direct = (_pool_regs(L, engine, pools[m], G).reshape(G, 16384) for m in ("1", "0"))
    bad = np.nonzero((part != direct).any(axis=1))[0]
    assert bad.size == 0, (bad.size, bad[:8].tolist(), np.unique(bad >> 12)[:8].tolist())
    for h in pools.values():
        L.rsk_hll_destroy(h)


@pytest.mark.parametrize("tm", [0, 1])
def test_grouped_partitioned_unaligned_group_ids(L, engine, orc, route, tm):
    """Device-resident pairs from element 1 on: the group ids are then not
    16-byte aligned (hll_gcount's scalar path) while the keys are; the
    partitioned add equals the direct kernel and the oracle."""
    from redisson_amd import _lib, devmem

    G, n = 5000, 2_000_003
    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n + 1)
    ks = k.keys_fixed(n, 16, offset=16).as_struct()
    pools = {}
    for mode in ("1", "0"):
        route(gpart=1 if mode == "1" else -1, gpart_tm=tm)
        h = _pool(L, engine, G)
        _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr + 4))
        pools[mode] = h
    part, direct = (_pool_regs(L, engine, pools[m], G) for m in ("1", "0"))
    assert np.array_equal(part, direct)
    ref = np.zeros(G * 16384, np.uint8)
    orc.hll_add_gen_grouped(ref, G, 0x5EED0006, 1, n)
    assert np.array_equal(part, ref)
    for h in pools.values():
        L.rsk_hll_destroy(h)
    g.free()
    k.free()


def test_grouped_partitioned_host_pairs_skip_out_of_range(L, engine, orc, route):
    """Host-resident pairs through the partitioned path: group ids >= G are
    ignored (as by the direct kernel), every other pair lands in its sketch;
    a second batch max-merges into the existing registers."""
    from redisson_amd import KeyBatch, _lib

    route(gpart=1)
    G, n = 100, 300_000
    rng = np.random.default_rng(7)
    keys = orc.gen_keys16(0x5EED0107, 0, n).reshape(-1, 16)
    groups = rng.integers(0, 130, n).astype(np.uint32)
    h = _pool(L, engine, G)
    for lo, hi in ((0, n // 3), (n // 3, n)):
        ks = KeyBatch.from_numpy(np.ascontiguousarray(keys[lo:hi])).as_struct()
        _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), np.ascontiguousarray(groups[lo:hi]).ctypes.data))
    got = _pool_regs(L, engine, h, G).reshape(G, 16384)
    for gid in range(G):
        sel = np.ascontiguousarray(keys[groups == gid])
        ref = np.zeros(16384, np.uint8)
        if sel.shape[0]:
            orc.hll_add(ref, sel.reshape(-1), None, 16, sel.shape[0])
        assert np.array_equal(got[gid], ref), gid
    L.rsk_hll_destroy(h)


def test_grouped_partitioned_pool_state_after_other_writers(L, engine, orc, route):
    """The partitioned add skips reading a pool known to be all zero (fresh or
    cleared): a PFADD into one sketch beforehand, and a clear afterwards, must
    both be honoured."""
    from redisson_amd import KeyBatch, _lib, devmem

    route(gpart=1)
    G, n = 64, 200_000
    h = _pool(L, engine, G)
    ka = orc.gen_keys16(0x5EED0200, 0, 5000)
    _add(L, h, KeyBatch.from_numpy(ka.reshape(-1, 16)), 5)
    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
    ks = k.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    grouped = np.zeros(G * 16384, np.uint8)
    orc.hll_add_gen_grouped(grouped, G, 0x5EED0006, 0, n)
    ref = grouped.copy()
    orc.hll_add(ref[5 * 16384:6 * 16384], ka, None, 16, 5000)
    assert np.array_equal(_pool_regs(L, engine, h, G), ref)
    _lib.check(L.rsk_hll_clear(h))
    assert not _pool_regs(L, engine, h, G).any()
    assert int(_count(L, h, [5])[0]) == 0
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    assert np.array_equal(_pool_regs(L, engine, h, G), grouped)
    # lazy clear completed by the grouped add itself: pairs only for sketches
    # 0..19, so rows 20..63 (full before the clear) must come back zero
    _lib.check(L.rsk_hll_clear(h))
    g2, k2 = devmem.gen_grouped(engine, 0x5EED0206, 20, 0, 100_000)
    ks2 = k2.keys_fixed(100_000, 16).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks2), g2.ptr))
    ref2 = np.zeros(G * 16384, np.uint8)
    orc.hll_add_gen_grouped(ref2[:20 * 16384], 20, 0x5EED0206, 0, 100_000)
    assert np.array_equal(_pool_regs(L, engine, h, G), ref2)
    cnt = _count(L, h, list(range(G)))
    assert cnt[20:].tolist() == [0] * (G - 20) and all(int(x) > 0 for x in cnt[:20])
    for b in (g, k, g2, k2):
        b.free()
    L.rsk_hll_destroy(h)


def test_batched_merge_and_union_follow_redis_order(L, engine, orc):
    """rsk_hll_merge_batch == PFMERGE dst src issued in order (chains and
    read-after-write inside one batch); rsk_hll_count_union_batch == PFCOUNT a b."""
    from redisson_amd import KeyBatch, _lib

    G = 64
    rng = np.random.default_rng(21)
    h = _pool(L, engine, G)
    r = orc.RedisModel()
    for g in range(0, G, 2):  # odd groups stay absent
        keys = orc.gen_keys16(0x5EED0100 + g, 0, int(rng.integers(1, 3000)))
        _add(L, h, KeyBatch.from_numpy(keys.reshape(-1, 16)), g)
        r.pfadd(str(g), *[keys[16 * i:16 * i + 16].tobytes() for i in range(keys.size // 16)])
    pairs = [(int(a), int(b)) for a, b in rng.integers(0, G, size=(300, 2))]
    pairs += [(1, 2), (3, 1), (5, 3), (2, 5)]  # chains through destinations
    d = np.array([p[0] for p in pairs], np.uint64)
    s = np.array([p[1] for p in pairs], np.uint64)
    _lib.check(L.rsk_hll_merge_batch(h, d.ctypes.data, s.ctypes.data, d.size))
    for a, b in pairs:
        r.pfmerge(str(a), str(b))
    for g in range(G):
        want = r.get(str(g))
        got = _regs(L, h, g)
        if want is None:
            assert not got.any()
        else:
            assert np.array_equal(got, orc.hll_decode(want)[1]), g
    members = rng.integers(0, G, size=(200, 3)).astype(np.uint64)
    out = np.zeros(200, np.uint64)
    _lib.check(L.rsk_hll_count_union_batch(h, members.ctypes.data, 3, 200, out.ctypes.data))
    for i in range(200):
        assert out[i] == r.pfcount(*[str(int(x)) for x in members[i]]), i
    cnt = _count(L, h, list(range(G)))
    assert [int(x) for x in cnt] == [r.pfcount(str(g)) for g in range(G)]


def test_c2_full_size_bit_exact(L, engine, orc):
    """BASELINE configs[1] at its full size: 1B 16-byte keys (device-generated
    C2 stream) give registers bit-identical to Redis PFADD arithmetic (the
    oracle, OpenMP over the same stream), and the exact PFCOUNT."""
    from redisson_amd import devmem

    n = 1_000_000_000
    t = devmem.gen_keys16(engine, SEED_C2, 0, n)
    h = _pool(L, engine)
    _add(L, h, t.keys_fixed(n, 16))
    t.free()
    ref = np.zeros(16384, np.uint8)
    orc.hll_add_gen16(ref, SEED_C2, 0, n, max(1, min(16, os.cpu_count() or 1)))
    got = _regs(L, h)
    assert np.array_equal(got, ref)
    assert int(_count(L, h, [0])[0]) == orc.hll_count_dense(ref)
    L.rsk_hll_destroy(h)


def test_c4_full_size_bit_exact(L, engine, orc):
    """BASELINE configs[3] at its per-GPU shard size: 1B variable-length keys
    (blob + offsets, 44 GB in HBM) through the LDS-staged kernel, bit-exact."""
    from redisson_amd import devmem

    n = 1_000_000_000
    blob, offs, tot = devmem.gen_varlen(engine, SEED_C4, 0, n)
    h = _pool(L, engine)
    _add(L, h, blob.keys_var(offs, n))
    blob.free()
    offs.free()
    ref = np.zeros(16384, np.uint8)
    orc.hll_add_gen_varlen(ref, SEED_C4, 0, n, max(1, min(16, os.cpu_count() or 1)))
    assert np.array_equal(_regs(L, h), ref)
    L.rsk_hll_destroy(h)


def _c5_stratified_sample(G: int, per_bin: int = 34, seed: int = 11) -> np.ndarray:
    """Sketch ids spread over the whole pool: from every coarse bin of the
    partitioned grouped add (4096 sketches, g >> 12) `per_bin` ids whose fine-
    bin slots (16 sketches, g & 15) cycle through all 16 positions and whose
    fine bins spread over the coarse bin; plus the pool's first and last ids."""
    rng = np.random.default_rng(seed)
    ids = [0, G - 1]
    for c in range((G + 4095) // 4096):
        lo, hi = c * 4096, min(G, (c + 1) * 4096)
        fines = (hi - lo + 15) // 16
        for j, fb in enumerate(rng.choice(fines, size=min(per_bin, fines), replace=False)):
            g = lo + 16 * int(fb) + j % 16
            ids.append(min(g, hi - 1))
    return np.unique(np.array(ids, np.uint64))


@pytest.mark.parametrize("tm", [1, 0, 2])  # 2: tile-major with 16384-record tiles (route gpart_tile)
def test_c5_full_size_group_sample_bit_exact(L, engine, orc, route, tm):
    """BASELINE configs[4] at its per-GPU size: 1M sketches, 500M (group, key)
    pairs through the grouped PFADD.  A stratified sample of >= 8192 sketches --
    ids from every coarse bin of the partitioned add and every slot of a fine
    bin, spread over the whole pool -- is bit-exact against the oracle over the
    whole pair stream, and PFCOUNT of the pool matches the oracle's estimator
    on them."""
    from redisson_amd import _lib, devmem

    route(gpart_tm=min(tm, 1), gpart_tile=int(tm == 2), gpart_poison=1)  # an unwritten fine-bin slot would raise a register to 63
    G, n = 1_000_000, 500_000_000
    sample = _c5_stratified_sample(G)
    gs = sample.size
    assert gs >= 8192 and np.unique(sample >> 12).size == (G + 4095) // 4096
    assert np.unique(sample & 15).size == 16
    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
    h = _pool(L, engine, G)
    ks = k.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    g.free()
    k.free()
    ref = np.zeros((gs, 16384), np.uint8)
    orc.hll_add_gen_grouped_ids(ref, G, sample, 0x5EED0006, 0, n, max(1, min(16, os.cpu_count() or 1)))
    base = L.rsk_hll_device_registers(h)
    bad = []
    for s, gid in enumerate(sample.tolist()):  # one 16 KiB row per sampled sketch
        row = np.zeros(16384, np.uint8)
        _lib.check(L.rsk_memcpy(engine.ctx, row.ctypes.data, ctypes.c_void_p(base + gid * 16384), 16384, 1))
        if not np.array_equal(row, ref[s]):
            bad.append(gid)
    assert not bad, (len(bad), bad[:10])
    cnt = _count(L, h, sample.tolist())
    chk = np.linspace(0, gs - 1, 128).astype(np.int64)
    assert [int(cnt[i]) for i in chk] == [orc.hll_count_dense(ref[i]) for i in chk]
    # the bench's batched countWith / mergeWith at full size: 10^5 ops over the
    # 1M sketches in one call each; the first 256 ops use only sampled sketches
    # (checked against the oracle), the rest draw from the whole pool.
    rng = np.random.default_rng(9)
    ops, chk = 100_000, 256
    slot = {int(gid): s for s, gid in enumerate(sample.tolist())}
    cw = rng.integers(0, G, size=(ops, 2), dtype=np.uint64)
    cw[:chk] = sample[rng.integers(0, gs, size=(chk, 2))]
    out = np.zeros(ops, np.uint64)
    _lib.check(L.rsk_hll_count_union_batch(h, cw.ctypes.data, 2, ops, out.ctypes.data))
    for i in range(chk):
        a, b = slot[int(cw[i, 0])], slot[int(cw[i, 1])]
        assert int(out[i]) == orc.hll_count_raw(np.maximum(ref[a], ref[b])), i
    perm = sample[rng.permutation(gs)]  # distinct sampled dst / src sketches
    rest = np.setdiff1d(np.arange(G, dtype=np.uint64), sample)
    md = rest[rng.integers(0, rest.size, size=ops)]
    ms = rest[rng.integers(0, rest.size, size=ops)]
    md[:chk], ms[:chk] = perm[:chk], perm[chk:2 * chk]
    _lib.check(L.rsk_hll_merge_batch(h, md.ctypes.data, ms.ctypes.data, ops))
    for i in range(0, chk, 8):
        d, sr = int(md[i]), int(ms[i])
        assert np.array_equal(_regs(L, h, d), np.maximum(ref[slot[d]], ref[slot[sr]])), i
        assert np.array_equal(_regs(L, h, sr), ref[slot[sr]]), i
    L.rsk_hll_destroy(h)


def _add_each(L, h, kb, i=0):
    from redisson_amd import _lib

    out = np.zeros(kb.n, np.uint8)
    ks = kb.as_struct()
    _lib.check(L.rsk_hll_add_each(h, i, ctypes.byref(ks), out.ctypes.data))
    return out


def test_add_each_skewed_runs(L, engine, orc):
    """Duplicate-heavy batches: one register's run spans many scan tiles."""
    from redisson_amd import KeyBatch

    # sequential Redis model on a small skewed batch (4 hot keys, 80 % of it)
    rng = np.random.default_rng(12)
    hot = [rng.integers(0, 256, 9, dtype=np.uint8).tobytes() for _ in range(4)]
    cold = [rng.integers(0, 256, 9, dtype=np.uint8).tobytes() for _ in range(6000)]
    keys = [hot[j] for j in rng.integers(0, 4, 24000)] + cold
    order = rng.permutation(len(keys))
    keys = [keys[j] for j in order]
    r = orc.RedisModel()
    want = [r.pfadd("k", e) for e in keys]
    h = _pool(L, engine)
    assert _add_each(L, h, KeyBatch.from_bytes_list(keys)).tolist() == want
    _, raw, _ = orc.hll_decode(r.get("k"))
    assert np.array_equal(_regs(L, h), raw)
    # 3M copies of one key: only the first can reply 1
    one = np.tile(orc.gen_keys16(SEED_C2, 5, 1), 3_000_000)
    h2 = _pool(L, engine)
    out = _add_each(L, h2, KeyBatch.from_numpy(one.reshape(-1, 16)))
    assert out[0] == 1 and int(out[1:].sum()) == 0
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, one[:16], None, 16, 1)
    assert np.array_equal(_regs(L, h2), ref)
    # 1M distinct keys four times over: passes 2-4 reply 0, pass 1 replies as a
    # fresh sketch does, registers as the oracle's
    n = 1 << 20
    k1 = orc.gen_keys16(SEED_C2, 0, n)
    h3, h4 = _pool(L, engine), _pool(L, engine)
    first = _add_each(L, h3, KeyBatch.from_numpy(k1.reshape(n, 16)))
    out4 = _add_each(L, h4, KeyBatch.from_numpy(np.tile(k1, 4).reshape(4 * n, 16)))
    assert np.array_equal(out4[:n], first) and int(out4[n:].sum()) == 0
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, k1, None, 16, n)
    assert np.array_equal(_regs(L, h4), ref) and np.array_equal(_regs(L, h3), ref)


def test_device_batch_with_host_output_is_rejected(L, engine, orc):
    """A pageable host pointer where the GPU would write (keys RSK_MEM_DEVICE)
    is refused with RSK_ERR_INVALID_ARG before any kernel runs."""
    from redisson_amd import _lib, devmem

    n = 1000
    t = devmem.gen_keys16(engine, SEED_C2, 0, n)
    ks = t.keys_fixed(n, 16).as_struct()
    host_out = np.zeros(n, np.uint8)
    h = _pool(L, engine)
    assert L.rsk_hll_add_each(h, 0, ctypes.byref(ks), host_out.ctypes.data) == _lib.RSK_ERR_INVALID_ARG
    b = ctypes.c_void_p()
    _lib.check(L.rsk_bloom_create(engine.ctx, 100000, 3, ctypes.byref(b)))
    assert L.rsk_bloom_contains(b, ctypes.byref(ks), host_out.ctypes.data) == _lib.RSK_ERR_INVALID_ARG
    assert L.rsk_bloom_add(b, ctypes.byref(ks), host_out.ctypes.data) == _lib.RSK_ERR_INVALID_ARG
    # host keys flagged as device-resident are refused too
    hk = orc.gen_keys16(SEED_C2, 0, n)
    bad = _lib.rsk_keys()
    bad.data, bad.offsets, bad.n, bad.fixed_len, bad.location = hk.ctypes.data, None, n, 16, _lib.RSK_MEM_DEVICE
    assert L.rsk_hll_add(h, 0, ctypes.byref(bad), None) == _lib.RSK_ERR_INVALID_ARG
    ex = ctypes.c_int(-1)
    _lib.check(L.rsk_hll_exists(h, 0, ctypes.byref(ex)))
    assert ex.value == 0  # a refused PFADD does not create the key
    empty = _lib.rsk_keys()
    empty.data, empty.offsets, empty.n, empty.fixed_len, empty.location = None, None, 0, 16, _lib.RSK_MEM_HOST
    changed = ctypes.c_uint8(7)
    _lib.check(L.rsk_hll_add(h, 0, ctypes.byref(empty), ctypes.byref(changed)))
    assert changed.value == 1  # PFADD key (no elements) on a missing key creates it: reply 1
    # and the context still works
    dout = devmem.DeviceBuffer.from_numpy(engine, np.zeros(n, np.uint8))
    _lib.check(L.rsk_bloom_contains(b, ctypes.byref(ks), dout.ptr))
    L.rsk_bloom_destroy(b)
    L.rsk_hll_destroy(h)


@pytest.mark.parametrize("n,branch", [(20_000, "linear"), (45_000, "bias"), (65_000, "bias"), (200_000, "raw")])
def test_count_estimator_branches(L, engine, orc, n, branch):
    # PFCOUNT on the GPU in each hllCount branch (linear counting, the 3.2.0
    # bias polynomial, raw) against a Python restatement that shares no code
    # with the oracle or the kernels (tests/redis_hllcount.py).
    from redis_hllcount import redis32_hllcount_raw

    from redisson_amd import KeyBatch

    keys = orc.gen_keys16(SEED_C2, 0, n)
    h = _pool(L, engine, 2)
    _add(L, h, KeyBatch.from_numpy(keys.reshape(n, 16)), 0)
    want, got_branch = redis32_hllcount_raw(_regs(L, h, 0))
    assert got_branch == branch
    assert int(_count(L, h, [0])[0]) == want  # single-key PFCOUNT (dense order)
    pools = (ctypes.c_void_p * 2)(h.value, h.value)
    ids = np.array([0, 1], np.uint64)  # sketch 1 empty: union == sketch 0 (raw order)
    out = np.zeros(1, np.uint64)
    from redisson_amd import _lib

    _lib.check(L.rsk_hll_count_union(pools, ids.ctypes.data, 2, out.ctypes.data))
    assert int(out[0]) == want
    L.rsk_hll_destroy(h)


@pytest.mark.parametrize("tm", [0, 1])
def test_zipf_stream_matches_oracle_and_partitioned_add(L, engine, orc, route, tm):
    """C5 Zipf(1.1) stress variant: the device generator equals the
    oracle's pair stream; the partitioned grouped add over it (one coarse bin
    holding most pairs, one fine bin a third of them) equals the direct kernel
    and the oracle over the whole pool."""
    from redisson_amd import _lib, devmem

    G, n = 20_000, 3_000_000
    g, k = devmem.gen_grouped_zipf(engine, 0x5EED0006, G, 1.1, 0, n)
    rg, rk = orc.gen_grouped_zipf(0x5EED0006, G, 1.1, 0, n)
    assert np.array_equal(g.to_numpy(np.uint32), rg) and np.array_equal(k.to_numpy(), rk)
    assert (rg == 0).mean() > 0.05  # skewed: rank 1 alone draws > 5 % of the pairs
    ks = k.keys_fixed(n, 16).as_struct()
    pools = {}
    for mode in ("1", "0"):
        route(gpart=1 if mode == "1" else -1, gpart_tm=tm)
        h = _pool(L, engine, G)
        _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
        pools[mode] = h
    g.free()
    k.free()
    part, direct = (_pool_regs(L, engine, pools[m], G) for m in ("1", "0"))
    assert np.array_equal(part, direct)
    ref = np.zeros(G * 16384, np.uint8)
    orc.hll_add_gen_grouped_zipf_subset(ref, G, G, 1.1, 0x5EED0006, 0, n, max(1, min(16, os.cpu_count() or 1)))
    assert np.array_equal(part, ref)
    # PFCOUNT of every sketch: estimated by the grouped add (split heavy bins excluded) or recomputed
    want = [orc.hll_count_dense(ref[i * 16384:(i + 1) * 16384]) for i in range(G)]
    assert _count(L, pools["1"], list(range(G))).tolist() == want
    for h in pools.values():
        L.rsk_hll_destroy(h)


def test_c5_zipf_full_size_hot_groups_bit_exact(L, engine, orc):
    """The Zipf(1.1) variant at the C5 per-GPU size (1M sketches, 500M pairs):
    the 1024 hottest sketches (about 60 % of all pairs) bit-exact against the
    oracle over the whole stream, and their PFCOUNTs."""
    from redisson_amd import _lib, devmem

    G, n, gs = 1_000_000, 500_000_000, 1024
    g, k = devmem.gen_grouped_zipf(engine, 0x5EED0006, G, 1.1, 0, n)
    h = _pool(L, engine, G)
    ks = k.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    g.free()
    k.free()
    ref = np.zeros((gs, 16384), np.uint8)
    orc.hll_add_gen_grouped_zipf_subset(ref, G, gs, 1.1, 0x5EED0006, 0, n, max(1, min(16, os.cpu_count() or 1)))
    got = np.zeros((gs, 16384), np.uint8)
    _lib.check(L.rsk_memcpy(engine.ctx, got.ctypes.data, L.rsk_hll_device_registers(h), got.nbytes, 1))
    assert np.array_equal(got, ref)
    cnt = _count(L, h, list(range(gs)))
    assert [int(c) for c in cnt[:64]] == [orc.hll_count_dense(ref[i]) for i in range(64)]
    L.rsk_hll_destroy(h)


def test_grouped_add_precomputed_counts_follow_later_writes(L, engine, orc, route):
    """The partitioned grouped add leaves every written row's PFCOUNT estimate
    for rsk_hll_count (no 16 KiB re-read); any later write to the pool (PFADD,
    PFMERGE, raw merge, import, clear, a second grouped add) must retire those
    estimates, and every count must equal the oracle's on the current registers."""
    from redisson_amd import KeyBatch, _lib, devmem

    route(gpart=1)
    G, n = 300, 600_000
    h = _pool(L, engine, G)
    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
    ks = k.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))

    def check_all():
        regs = _pool_regs(L, engine, h, G).reshape(G, 16384)
        want = [orc.hll_count_dense(regs[i]) for i in range(G)]
        assert _count(L, h, list(range(G))).tolist() == want
        assert _count(L, h, list(range(G))).tolist() == want  # second call: from the card cache
        return regs

    check_all()
    # each writer, then the counts of the whole pool again
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))  # idempotent re-add: fresh estimates
    check_all()
    ka = orc.gen_keys16(0x5EED0300, 0, 40_000)
    _add(L, h, KeyBatch.from_numpy(ka.reshape(-1, 16)), 7)
    regs = check_all()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    pools = (ctypes.c_void_p * 1)(h.value)
    srcs = (ctypes.c_uint64 * 1)(7)
    _lib.check(L.rsk_hll_merge(h, 11, pools, srcs, 1))
    check_all()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    raw = np.full(16384, 9, np.uint8)
    _lib.check(L.rsk_hll_merge_raw(h, 13, raw.ctypes.data, _lib.RSK_MEM_HOST))
    check_all()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    sp = orc.hll_encode_sparse(regs[3])
    b = (ctypes.c_uint8 * len(sp)).from_buffer_copy(sp)
    _lib.check(L.rsk_hll_import_redis(h, 17, b, len(sp)))
    check_all()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    _lib.check(L.rsk_hll_clear(h))
    assert _count(L, h, list(range(G))).tolist() == [0] * G
    # a second grouped add over a different stream after the clear
    g2, k2 = devmem.gen_grouped(engine, 0x5EED0306, G, 0, n)
    ks2 = k2.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks2), g2.ptr))
    ref = np.zeros(G * 16384, np.uint8)
    orc.hll_add_gen_grouped(ref, G, 0x5EED0306, 0, n)
    assert np.array_equal(check_all().reshape(-1), ref)
    for x in (g, k, g2, k2):
        x.free()
    L.rsk_hll_destroy(h)


def _export(L, h, i):
    from redisson_amd import _lib

    buf = (ctypes.c_uint8 * 12304)()
    n = ctypes.c_size_t()
    _lib.check(L.rsk_hll_export_redis(h, i, buf, 12304, ctypes.byref(n)))
    return bytes(buf[: n.value])


def test_export_follows_redis_encoding(L, engine, orc):
    """GET of a key as Redis 3.2.0 would hold it: sparse while the registers fit
    (values <= 32, <= 3000 bytes with the header), dense once promoted (for
    good), after PFMERGE (destination converted) and after SET of a dense
    string; byte-identical to the Redis model's canonical sparse form."""
    from redisson_amd import KeyBatch, _lib

    r = orc.RedisModel()
    h = _pool(L, engine, 4)
    keys = orc.gen_keys16(SEED_C2, 0, 4000).reshape(-1, 16)
    empty = np.zeros((0, 16), np.uint8)
    _add(L, h, KeyBatch.from_numpy(empty), 0)  # PFADD k (no elements): created, sparse XZERO
    r.pfadd("k")
    assert _export(L, h, 0) == r.get("k") and _export(L, h, 0)[4] == 1
    done = 0
    for upto in (1, 10, 100, 300, 600, 1200, 4000):
        batch = keys[done:upto]
        _add(L, h, KeyBatch.from_numpy(batch), 0)
        r.pfadd("k", *[bytes(x) for x in batch])
        done = upto
        s = _export(L, h, 0)
        assert s == r.get("k"), upto
        if upto in (100, 300):
            assert int(_count(L, h, [0])[0]) == r.pfcount("k")  # card cache refreshed, then read back out
            assert _export(L, h, 0) == r.get("k")
    assert _export(L, h, 0)[4] == 0  # 4000 keys: promoted to dense
    # PFMERGE destination: dense even when small
    _add(L, h, KeyBatch.from_numpy(keys[:5]), 1)
    r.pfadd("a", *[bytes(x) for x in keys[:5]])
    pools = (ctypes.c_void_p * 1)(h.value)
    src = (ctypes.c_uint64 * 1)(1)
    _lib.check(L.rsk_hll_merge(h, 2, pools, src, 1))
    r.pfmerge("m", "a")
    assert _export(L, h, 2) == r.get("m") and _export(L, h, 2)[4] == 0
    # SET of a sparse string keeps it sparse; of a dense one, dense
    sp = r.get("a")
    b = (ctypes.c_uint8 * len(sp)).from_buffer_copy(sp)
    _lib.check(L.rsk_hll_import_redis(h, 3, b, len(sp)))
    assert _export(L, h, 3) == sp
    dn = r.get("m")
    b = (ctypes.c_uint8 * len(dn)).from_buffer_copy(dn)
    _lib.check(L.rsk_hll_import_redis(h, 3, b, len(dn)))
    assert _export(L, h, 3)[4] == 0
    _lib.check(L.rsk_hll_delete(h, 3))  # DEL: a new key starts sparse again
    _add(L, h, KeyBatch.from_numpy(keys[:3]), 3)
    assert _export(L, h, 3)[4] == 1
    L.rsk_hll_destroy(h)


@pytest.mark.parametrize("zipf", [0.0, 1.1])
def test_c5_full_size_every_sketch_bit_exact(L, engine, orc, zipf):
    """BASELINE configs[4] at its per-GPU size (1M sketches, 500M pairs; uniform
    and the Zipf(1.1) stress variant): EVERY sketch of the pool bit-exact
    against the oracle over the whole pair stream -- 16 GB of registers
    compared row by row (the oracle on up to 16 cores, each owning a range of
    the groups) -- and PFCOUNT of an evenly spread sample of 1024 sketches."""
    from redisson_amd import _lib, devmem

    G, n, seed = 1_000_000, 500_000_000, 0x5EED0006
    thr = max(1, min(16, os.cpu_count() or 1))
    if zipf:
        g, k = devmem.gen_grouped_zipf(engine, seed, G, zipf, 0, n)
    else:
        g, k = devmem.gen_grouped(engine, seed, G, 0, n)
    h = _pool(L, engine, G)
    ks = k.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), g.ptr))
    g.free()
    k.free()
    groups = orc.gen_grouped_zipf_groups(seed, G, zipf, 0, n, thr) if zipf else orc.gen_grouped_groups(seed, G, 0, n, thr)
    ref = np.zeros((G, 16384), np.uint8)
    orc.hll_add_keys_by_groups(ref, G, groups, seed, 0, thr)
    del groups
    base = L.rsk_hll_device_registers(h)
    chunk = 65536
    buf = np.empty((chunk, 16384), np.uint8)
    bad = []
    for lo in range(0, G, chunk):
        m = min(chunk, G - lo)
        _lib.check(L.rsk_memcpy(engine.ctx, buf.ctypes.data, ctypes.c_void_p(base + lo * 16384), m * 16384, 1))
        diff = np.nonzero((buf[:m] != ref[lo:lo + m]).any(1))[0]
        bad.extend((diff + lo)[:16].tolist())
    assert not bad, (len(bad), bad[:16])
    sample = np.linspace(0, G - 1, 1024).astype(np.int64)
    cnt = _count(L, h, sample.tolist())
    assert [int(c) for c in cnt] == [orc.hll_count_dense(ref[i]) for i in sample]
    L.rsk_hll_destroy(h)
    _lib.check(L.rsk_trim(engine.ctx))


def test_large_count_mixes_cache_precomputed_and_recomputed(L, engine, orc, route):
    """A PFCOUNT batch of >= 4096 ids takes the two-phase count (a lane per
    sketch answers from the card cache or the grouped add's precomputed
    estimate and lists the rest, then a wave per listed sketch): on a pool
    holding all three states -- cached by an earlier count, stamped by the
    partitioned add, invalidated by a merge, a raw register write and a
    per-key add -- and with duplicate ids, it equals the one-wave-per-sketch
    count (batches under 4096) on an identical pool and the oracle's count of
    the registers."""
    from redisson_amd import KeyBatch, devmem
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    route(gpart=1)
    G, n = 20000, 4_000_000
    rng = np.random.default_rng(41)
    regs = rng.integers(0, 9, 16384).astype(np.uint8)
    extra = orc.gen_keys16(SEED_C2 + 77, 0, 3000).reshape(3000, 16)
    pools = []
    for _ in range(2):
        g, k = devmem.gen_grouped(engine, 0x5EED0041, G, 0, n)
        p = GroupedHyperLogLog(engine, G)
        p.add(k.keys_fixed(n, 16), g)
        g.free()
        k.free()
        p.count(np.arange(0, 1000, dtype=np.uint64))  # cached
        p.mergeWith(np.arange(1000, 2000, dtype=np.uint64), np.arange(5000, 6000, dtype=np.uint64))
        _lib_merge_raw(L, p.pool, 2500, regs)
        _add(L, p.pool, KeyBatch.from_numpy(extra), 3000)
        pools.append(p)
    ids = np.concatenate([np.arange(G, dtype=np.uint64), np.array([7, 1500, 2500, 3000, 19999], np.uint64)])
    every = pools[0].count().copy()  # (no id list: the whole pool, two-phase)
    big = pools[0].count(ids)  # (now from the cache, duplicates included)
    small = np.concatenate([pools[1].count(ids[i:i + 4000]) for i in range(0, ids.size, 4000)])
    assert np.array_equal(every, small[:G])
    assert np.array_equal(big, small)
    for gid in (0, 999, 1000, 1999, 2500, 3000, 5000, 19999):
        assert int(big[gid]) == orc.hll_count_dense(pools[0].registers(gid)), gid
    for p in pools:
        p.close()


def _lib_merge_raw(L, h, i, regs):
    from redisson_amd import _lib

    _lib.check(L.rsk_hll_merge_raw(h, i, regs.ctypes.data, _lib.RSK_MEM_HOST))
