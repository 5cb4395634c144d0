"""RBloomFilter.add() replies (RedissonBloomFilter.java:100-107) through the
partitioned first-probe pipeline (rsk_bloom_reply.hip): replies and bit strings
against the oracle's sequential SETBITs, and against the sort path."""
import ctypes

import numpy as np
import pytest

from test_gpu_bloom import _add, _bits, _filter


@pytest.fixture(scope="module")
def L():
    from redisson_amd import _lib

    return _lib.load()


def test_sampled_reply_oracle_matches_sequential(orc):
    """The sampled full-size reply oracle (hash table of the sample's bits, min
    sequence number over the whole stream) equals the sequential SETBIT oracle."""
    size, k, n = 200003, 7, 30000
    keys = orc.gen_keys16(0x5EED0003, 0, n)
    bits = np.zeros((size + 7) // 8, np.uint8)
    want = orc.bloom_add_batch(bits, size, k, keys, None, 16, n)
    sample = np.unique(np.random.default_rng(1).integers(0, n, 3000)).astype(np.uint64)
    got = orc.bloom_add_replies_sample_gen16_mt(size, k, 0x5EED0003, n, sample, 4)
    assert np.array_equal(got, want[sample.astype(np.int64)])
    assert 0 < got.sum() < got.size  # both answers occur at this fill


CASES = [(1, 2, 5000), (729, 5, 20000), (95851, 7, 50000), (1000003, 1, 50000), (1000003, 3, 200000), (1000003, 33, 20000),
         (19170117, 7, 300000), (157298745, 7, 400000), (157298745, 9, 200000), (157298745, 16, 150000),
         (4014142460, 8, 600000)]
KNOBS = ["reply=1", "reply=1,reply_chunk=300000", "reply=1,sa_tiny=1", "reply=1,sa_parts=13", "reply=1,sa_parts=1",
         "reply=1,reply_v=3", "reply=1,reply_v=6", "reply=1,reply_s=4,reply_u=4", "reply=1,reply_s=1,reply_u=1"]


@pytest.mark.gpu
@pytest.mark.parametrize("size,k,n", CASES)
@pytest.mark.parametrize("knobs", KNOBS)
def test_replies_parity(L, engine, orc, route, size, k, n, knobs):
    """Forced on at every size: one partition level (<= 256 slices) and two
    (301 and 7,657 slices), k in {1, 2, 3, 5, 7, 8, 9, 16} (33: the sort path); many chunks (each
    answered against the filter the earlier ones left); sub-regions too small
    (the chunk falls back to the sort path); rp2 with 13 parts per coarse bin
    and with one; the kernel forms (rp2 tiles of 12288 records, rp_tapply on
    one or four steps of segment loads per fold, 1 or 4 gather chains per lane).  A second batch of variable-length
    keys repeats keys of the first and of itself (bits already set before the
    batch, first probes inside it)."""
    from redisson_amd import KeyBatch

    route(knobs)
    keys = orc.gen_keys16(0x5EED0003, 0, n)
    b = _filter(L, engine, size, k)
    got = _add(L, b, KeyBatch.from_numpy(keys.reshape(-1, 16)))
    ref = np.zeros((size + 7) // 8, np.uint8)
    want = orc.bloom_add_batch(ref, size, k, keys, None, 16, n)
    assert np.array_equal(got, want)
    assert np.array_equal(_bits(L, b, size), ref)
    rng = np.random.default_rng(k + n)
    vk = [rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes() for _ in range(4000)]
    vk += vk[:1000] + [b""] + [bytes(keys[16 * i: 16 * i + 16]) for i in range(0, min(n, 3000), 3)]
    rng.shuffle(vk)
    got = _add(L, b, KeyBatch.from_bytes_list(vk))
    blob, offs = orc.pack_keys(vk)
    want = orc.bloom_add_batch(ref, size, k, blob, offs)
    assert np.array_equal(got, want)
    assert np.array_equal(_bits(L, b, size), ref)
    L.rsk_bloom_destroy(b)


@pytest.mark.gpu
@pytest.mark.parametrize("knobs", KNOBS[:2])
def test_replies_skewed_keys(L, engine, orc, route, knobs):
    """One key repeated 300,000 times among distinct ones: only its first copy
    can answer true; every probe of the copies lands on the same k bits."""
    from redisson_amd import KeyBatch

    route(knobs)
    size, k = 157298745, 7
    base = orc.gen_keys16(0x5EED0003, 0, 1000).reshape(-1, 16)
    keys = np.concatenate([base[1:500], np.repeat(base[:1], 300000, axis=0), base[500:]]).reshape(-1)
    n = keys.size // 16
    b = _filter(L, engine, size, k)
    got = _add(L, b, KeyBatch.from_numpy(keys.reshape(-1, 16)))
    ref = np.zeros((size + 7) // 8, np.uint8)
    want = orc.bloom_add_batch(ref, size, k, keys, None, 16, n)
    assert np.array_equal(got, want)
    assert want[499] == 1 and not want[500:300499].any()
    assert np.array_equal(_bits(L, b, size), ref)
    L.rsk_bloom_destroy(b)


@pytest.mark.gpu
@pytest.mark.parametrize("dup", [False, True])
def test_replies_pending_groups(L, engine, orc, route, dup):
    """Bits probed more than once by the key group that probed them first:
    in a 2M-bit filter every 2048-key group has ~50 such bits, and a key whose
    only candidate bits are among them stays pending until its workgroup has
    scanned the group again (resolved in LDS, no fallback).  With every key
    repeated right after itself each group holds ~1000 pending keys, more than
    its LDS tables take: the chunk's bits are restored from T and the sort path
    answers it.  Both against the sequential SETBITs."""
    from redisson_amd import KeyBatch, _lib

    route("reply=1")
    size, k, n = 2000003, 7, 100000
    keys = orc.gen_keys16(0x5EED0007, 0, n).reshape(-1, 16)
    if dup:
        keys = np.repeat(keys[: n // 2], 2, axis=0)
    keys = np.ascontiguousarray(keys).reshape(-1)
    ref = np.zeros((size + 7) // 8, np.uint8)
    ref[:1000] = 0xA5  # bits set before the batch: no probe on them answers true
    b = _filter(L, engine, size, k)
    _lib.check(L.rsk_bloom_import_bits(b, ref.ctypes.data, ref.size))
    pg0, fb0 = engine.reply_stats()
    got = _add(L, b, KeyBatch.from_numpy(keys.reshape(-1, 16)))
    want = orc.bloom_add_batch(ref, size, k, keys, None, 16, keys.size // 16)
    assert np.array_equal(got, want)
    assert np.array_equal(_bits(L, b, size), ref)
    pg1, fb1 = engine.reply_stats()
    if dup:
        assert fb1 > fb0  # answered by the fallback
    else:
        assert pg1 > pg0 and fb1 == fb0  # pending probes resolved in LDS
    L.rsk_bloom_destroy(b)


@pytest.mark.gpu
def test_replies_match_sort_path_c3_filter(L, engine, route):
    """At the C3 filter size (9,585,058,377 bits, k = 7: 143 coarse bins x 128
    slices x 16 blocks) 20M device-resident keys give the same replies and bit
    string through the partitioned pipeline and through the sort path, into an
    empty filter and again into the filled one."""
    from redisson_amd import _lib, devmem

    size, k, n = 9585058377, 7, 20_000_000
    ins = devmem.gen_keys16(engine, 0x5EED0003, 0, n)
    ks = ins.keys_fixed(n, 16).as_struct()
    half = ins.keys_fixed(n // 2, 16).as_struct()
    res = {}
    for mode in ("1", "0"):
        route(reply=1 if mode == "1" else -1)
        f = _filter(L, engine, size, k)
        out = devmem.DeviceBuffer(engine, n)
        _lib.check(L.rsk_bloom_add(f, ctypes.byref(ks), out.ptr))
        first = out.to_numpy()
        _lib.check(L.rsk_bloom_add(f, ctypes.byref(half), out.ptr))
        again = out.to_numpy()[: n // 2]
        bc = ctypes.c_uint64()
        _lib.check(L.rsk_bloom_bitcount(f, ctypes.byref(bc)))
        res[mode] = (first, again, bc.value, f)
        out.free()
    assert np.array_equal(res["1"][0], res["0"][0])
    assert res["1"][0].mean() > 0.99  # 20M keys in a filter sized for 1B: nearly all new
    assert not res["1"][1].any() and not res["0"][1].any()  # re-adding answers false
    assert res["1"][2] == res["0"][2]
    nbytes = (size + 7) // 8
    _lib.check(L.rsk_bloom_or_bits(res["1"][3], L.rsk_bloom_device_bits(res["0"][3]), nbytes, _lib.RSK_MEM_DEVICE))
    bc = ctypes.c_uint64()
    _lib.check(L.rsk_bloom_bitcount(res["1"][3], ctypes.byref(bc)))
    assert bc.value == res["0"][2]  # OR changes nothing: equal bit strings
    for r in res.values():
        L.rsk_bloom_destroy(r[3])
    ins.free()


@pytest.mark.gpu
def test_c3_full_size_replies(L, engine, orc, route):
    """BASELINE configs[2] with the reference's add() semantics at full size:
    1B keys in one add() call into the 9,585,058,377-bit filter (k = 7, one
    chunk); all 1B replies equal the sort path's (an independent algorithm: a
    stable radix sort of (bit, sequence)), 200,000 sampled replies equal the
    oracle's (exact minimum sequence number over the whole stream for the
    sample's bits), and the bit string equals the reply-less insert's."""
    import os

    from redisson_amd import _lib, devmem

    n, size, k = 1_000_000_000, 9585058377, 7
    threads = max(1, min(16, os.cpu_count() or 1))
    ins = devmem.gen_keys16(engine, 0x5EED0003, 0, n)
    ks = ins.keys_fixed(n, 16).as_struct()
    b = _filter(L, engine, size, k)
    out = devmem.DeviceBuffer(engine, n)
    pg0, fb0 = engine.reply_stats()
    _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), out.ptr))
    got = out.to_numpy()
    pg1, fb1 = engine.reply_stats()
    assert fb1 == fb0 and pg1 > pg0  # the group-tag pipeline answered, pending groups resolved in LDS
    route(reply=-1)  # the sort path, into a fresh filter
    srt = _filter(L, engine, size, k)
    _lib.check(L.rsk_bloom_add(srt, ctypes.byref(ks), out.ptr))
    assert np.array_equal(got, out.to_numpy())
    L.rsk_bloom_destroy(srt)
    route("reset=0")
    out.free()
    plain = _filter(L, engine, size, k)
    _lib.check(L.rsk_bloom_add(plain, ctypes.byref(ks), None))
    ins.free()
    bc_a, bc_p, bc_b = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(L.rsk_bloom_bitcount(b, ctypes.byref(bc_a)))
    _lib.check(L.rsk_bloom_bitcount(plain, ctypes.byref(bc_p)))
    _lib.check(L.rsk_bloom_or_bits(b, L.rsk_bloom_device_bits(plain), (size + 7) // 8, _lib.RSK_MEM_DEVICE))
    _lib.check(L.rsk_bloom_bitcount(b, ctypes.byref(bc_b)))
    assert bc_a.value == bc_p.value == bc_b.value  # equal counts, OR changes nothing: equal bit strings
    L.rsk_bloom_destroy(b)
    L.rsk_bloom_destroy(plain)
    rng = np.random.default_rng(0xC3)
    sample = np.unique(np.concatenate([rng.integers(0, n, 200_000), np.arange(1000),
                                       np.arange(n - 1000, n)])).astype(np.uint64)
    want = orc.bloom_add_replies_sample_gen16_mt(size, k, 0x5EED0003, n, sample, threads)
    assert np.array_equal(got[sample.astype(np.int64)], want)
    frac = float(got.mean())
    assert 0.9 < frac < 1.0  # distinct keys: false only when all 6 first probes were taken
