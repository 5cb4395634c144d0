"""Pin the CPU oracle before trusting it (CPU only).

Every check here compares the oracle against something it was not derived
from: published known answers for the hash functions, an independent XXH64
implementation, and the expectations of the reference's own JUnit tests.
"""
import json
import os
import struct

import numpy as np
import pytest
from redis_hllcount import redis32_hllcount_raw

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden.json")


def test_murmur64a_smhasher_verification(orc):
    # SMHasher VerificationTest: keys {0..i-1} hashed with seed 256-i, the
    # concatenated hashes hashed with seed 0; "Murmur2B" = 0x1F0D3804.
    L = orc.lib()
    key = bytearray(256)
    hashes = bytearray()
    for i in range(256):
        key[i] = i
        hashes += struct.pack("<Q", L.orc_murmur64a(bytes(key[:i]), i, 256 - i))
    final = L.orc_murmur64a(bytes(hashes), len(hashes), 0)
    assert final & 0xFFFFFFFF == 0x1F0D3804


def test_xxh64_matches_python_xxhash(orc):
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(1)
    for n in list(range(0, 100)) + [127, 128, 129, 1000, 4096]:
        for _ in range(3):
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert orc.xxh64(b) == xxhash.xxh64_intdigest(b, 0)
    assert orc.xxh64(b"") == 0xEF46DB3751D8E999
    assert orc.xxh64(b'"123"') == 0xAE40987216FED2E5


def _s64(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def test_farmhash_na_guava_known_answers(orc):
    # Guava FarmHashFingerprint64Test.testReallySimpleFingerprints
    # (Fingerprint64 == farmhashna::Hash64): lengths 4, 32 and 256.
    assert _s64(orc.farmhash_na64(b"test")) == 8581389452482819506
    assert _s64(orc.farmhash_na64(b"test" * 8)) == -4196240717365766262
    assert _s64(orc.farmhash_na64(b"test" * 64)) == 3500507768004279527
    assert orc.farmhash_na64(b"") == 0x9AE16A3B2F90404F  # k2


def test_farmhash_uo_equals_na_up_to_64(orc):
    for n in range(0, 65):
        b = bytes((i * 7 + 3) & 0xFF for i in range(n))
        assert orc.farmhash_uo64(b) == orc.farmhash_na64(b)


def test_reference_hll_junit_add(orc):
    # RedissonHyperLogLogTest.testAdd: JSON codec, Integer 1,2,3 -> b"1".. ; count()==3
    r = orc.RedisModel()
    for e in (b"1", b"2", b"3"):
        r.pfadd("log", e)
    assert r.pfcount("log") == 3


def test_reference_hll_junit_merge(orc):
    # RedissonHyperLogLogTest.testMerge
    r = orc.RedisModel()
    j = lambda s: ('"%s"' % s).encode()  # noqa: E731
    assert [r.pfadd("hll1", j(s)) for s in ("foo", "bar", "zap", "a")] == [1, 1, 1, 1]
    assert [r.pfadd("hll2", j(s)) for s in ("a", "b", "c", "foo", "c")] == [1, 1, 1, 1, 0]
    r.pfmerge("hll3", "hll1", "hll2")
    assert r.pfcount("hll3") == 6


def test_reference_bloom_junit_config(orc):
    # RedissonBloomFilterTest.testConfig: tryInit(100, 0.03) -> size 729, k 5
    size = orc.bloom_optimal_bits(100, 0.03)
    assert size == 729 and orc.bloom_optimal_k(100, size) == 5
    # RedissonBloomFilterTest.test: tryInit(550000000, 0.03) fits under MAX_SIZE
    size = orc.bloom_optimal_bits(550000000, 0.03)
    assert size == 4014142460 and size <= 2147483647 * 2
    assert orc.bloom_optimal_k(550000000, size) == 5


def test_reference_bloom_junit_sequence(orc):
    # RedissonBloomFilterTest.test, replayed through the oracle Redis model.
    r = orc.RedisModel()
    f = orc.OracleBloomFilter(r, "filter", lambda s: ('"%s"' % s).encode())
    assert f.try_init(550000000, 0.03)
    assert not f.contains("123")
    assert f.add("123")
    assert f.contains("123")
    assert not f.add("123")
    assert f.count() == 1
    s = "hflgs;jl;ao1-32471320o31803-24"
    assert not f.contains(s)
    assert f.add(s)
    assert f.contains(s)
    assert f.count() == 2


def test_reference_bloom_junit_init(orc):
    r = orc.RedisModel()
    f = orc.OracleBloomFilter(r, "filter", lambda s: s.encode())
    assert f.try_init(55000000, 0.03)
    assert not f.try_init(55000001, 0.03)
    r.delete("filter", "{filter}__config")
    assert f.try_init(55000001, 0.03)


def test_bloom_max_size(orc):
    # 1B @ 1% exceeds MAX_SIZE: the reference throws (RedissonBloomFilter.java:226-227)
    assert orc.bloom_optimal_bits(10 ** 9, 0.01) == 9585058377
    assert orc.bloom_optimal_bits(4 * 10 ** 8, 0.01) == 3834023350


def test_bloom_k1_semantics(orc):
    # k == 1: subList(1, size-1) is empty -> add() always False, contains() always True
    bits = np.zeros(16, np.uint8)
    keys = np.frombuffer(b"abcdefgh" * 4, np.uint8).copy()
    added = orc.bloom_add_batch(bits, 100, 1, keys, None, 8, 4)
    assert not added.any()
    assert orc.bloom_contains_batch(np.zeros(16, np.uint8), 100, 1, keys, None, 8, 4).all()


def test_hll_sparse_dense_roundtrip(orc):
    regs = np.zeros(orc.REGISTERS, np.uint8)
    orc.hll_add_gen16(regs, 0x5EED0002, 0, 3000)
    sp = orc.hll_encode_sparse(regs)
    de = orc.hll_encode_dense(regs)
    assert len(de) == orc.DENSE_SIZE
    for s in (sp, de):
        rc, raw, enc = orc.hll_decode(s)
        assert rc == 0 and np.array_equal(raw, regs)
    # sparse and dense PFCOUNT agree (exact sums)
    assert orc.hll_count_string(sp)[1] == orc.hll_count_string(de)[1] == orc.hll_count_raw(regs)


def test_hll_decode_rejects(orc):
    assert orc.hll_decode(b"HYLL")[0] == -1                         # short
    assert orc.hll_decode(b"HYLX" + b"\0" * 12304)[0] == -1          # magic
    assert orc.hll_decode(b"HYLL\x00" + b"\0" * 100)[0] == -1        # dense wrong length
    assert orc.hll_decode(b"HYLL\x02" + b"\0" * 11)[0] == -1         # encoding > 1
    bad = b"HYLL\x01" + b"\0" * 11 + bytes([0x7F, 0xFE])              # XZERO 16383, total != 16384
    assert orc.hll_decode(bad)[0] == -2


def test_golden_fixtures_reproduce(orc):
    g = json.load(open(GOLDEN))
    xs = [bytes.fromhex(h) for h in g["hash_inputs_hex"]]
    assert ["%016x" % orc.murmur64a(x) for x in xs] == g["murmur64a_seed_adc83b19"]
    assert ["%016x" % orc.xxh64(x) for x in xs] == g["xxh64_seed0"]
    assert ["%016x" % orc.farmhash_uo64(x) for x in xs] == g["farmhash_uo64"]
    for n, p, size, k in g["bloom_params"]:
        assert orc.bloom_optimal_bits(n, p) == size and orc.bloom_optimal_k(n, size) == k
    regs = np.zeros(orc.REGISTERS, np.uint8)
    orc.hll_add_gen16(regs, 0x5EED0002, 0, 20000)
    assert regs.tobytes().hex() == g["hll"]["c2_20000"]["registers_hex"]
    assert orc.hll_count_dense(regs) == g["hll"]["c2_20000"]["count_dense"]


def test_multithreaded_cpu_baseline_matches_sequential(orc):
    # bench.py's all-cores CPU figure must compute the same registers as the 1-core port
    keys = orc.gen_keys16(0x5EED0002, 0, 200_000)
    seq = np.zeros(orc.REGISTERS, np.uint8)
    orc.hll_add(seq, keys, None, 16, 200_000)
    for threads in (1, 3, 8):
        mt = np.zeros(orc.REGISTERS, np.uint8)
        orc.hll_add_fixed_mt(mt, keys, 16, 200_000, threads)
        assert np.array_equal(mt, seq), threads


def test_c3_query_stream_fresh_keys_are_fresh(orc):
    # C3 queries: r&1 -> an inserted key, else a fresh key from a state range the
    # insert stream never reaches; the fresh half shows the filter's ~1% FP rate.
    n = 200_000
    size = orc.bloom_optimal_bits(n, 0.01)
    k = orc.bloom_optimal_k(n, size)
    bits = np.zeros((size + 7) // 8, np.uint8)
    orc.bloom_add_batch(bits, size, k, orc.gen_keys16(0x5EED0003, 0, n), None, 16, n, want=False)
    q = orc.gen_queries16(0x5EED0004, 0x5EED0003, n, 0, n)
    got = orc.bloom_contains_batch(bits, size, k, q, None, 16, n).astype(bool)
    member = np.array([orc.splitmix64(0x5EED0004 + 3 * i) & 1 for i in range(n)], bool)
    assert got[member].all()
    assert 0.40 < member.mean() < 0.60
    assert got[~member].mean() < 0.03


def test_varlen_stream_oracle_forms_agree(orc):
    # the on-the-fly C4 oracle (used for the full-size GPU check) equals the packed-blob one
    blob, offs = orc.gen_varlen(0x5EED0005, 1000, 50_000)
    a = np.zeros(orc.REGISTERS, np.uint8)
    orc.hll_add(a, blob, offs)
    for threads in (1, 4):
        b = np.zeros(orc.REGISTERS, np.uint8)
        orc.hll_add_gen_varlen(b, 0x5EED0005, 1000, 50_000, threads)
        assert np.array_equal(a, b), threads


def test_bloom_stream_oracle_forms_agree(orc):
    # the OpenMP C3 oracle twins (full-size GPU check) equal the sequential batch forms
    n, size, k = 30_000, 287_552, 7
    keys = orc.gen_keys16(0x5EED0003, 0, n)
    a = np.zeros((size + 7) // 8, np.uint8)
    orc.bloom_add_batch(a, size, k, keys, None, 16, n, want=False)
    b = np.zeros_like(a)
    orc.bloom_add_gen16_mt(b, size, k, 0x5EED0003, 0, n, 4)
    assert np.array_equal(a, b)
    q = orc.gen_queries16(0x5EED0004, 0x5EED0003, n, 0, n)
    want = orc.bloom_contains_batch(a, size, k, q, None, 16, n)
    got = np.zeros(n, np.uint8)
    assert orc.bloom_contains_gen_queries_mt(a, size, k, 0x5EED0004, 0x5EED0003, n, 0, n, got, 4) == int(want.sum())
    assert np.array_equal(got, want)


def test_grouped_subset_oracle_matches_full(orc):
    G, n = 50, 20_000
    full = np.zeros((G, orc.REGISTERS), np.uint8)
    orc.hll_add_gen_grouped(full, G, 0x5EED0006, 0, n)
    for threads in (1, 3):
        sub = np.zeros((7, orc.REGISTERS), np.uint8)
        orc.hll_add_gen_grouped_subset(sub, G, 7, 0x5EED0006, 0, n, threads)
        assert np.array_equal(sub, full[:7]), threads
    ids = np.array([49, 3, 17, 0, 32], np.uint64)
    for threads in (1, 4):
        sub = np.zeros((ids.size, orc.REGISTERS), np.uint8)
        orc.hll_add_gen_grouped_ids(sub, G, ids, 0x5EED0006, 0, n, threads)
        assert np.array_equal(sub, full[ids.astype(np.int64)]), threads


def test_hash_to_base64_cpu_form_shape(orc):
    # the CPU form the GPU misc/Hash test compares with: 16 bytes -> 24 Base64 chars, "==" dropped
    import base64
    import struct

    import xxhash

    s = base64.b64encode(struct.pack(">QQ", orc.farmhash_uo64(b"test"), xxhash.xxh64_intdigest(b"test", 0))).decode()
    assert len(s) == 24 and s.endswith("==")


def _absl_cityhash64():
    """absl's CityHash64 (CityHash v1.1, absl/hash/internal/city.cc) as exported by
    the pyarrow wheel in this image: an implementation independent of ours."""
    import ctypes
    import glob
    import importlib.util

    spec = importlib.util.find_spec("pyarrow")
    if spec is None or not spec.submodule_search_locations:
        pytest.skip("pyarrow not importable")
    for path in sorted(glob.glob(os.path.join(list(spec.submodule_search_locations)[0], "libarrow_compute.so*"))):
        try:
            lib = ctypes.CDLL(path)
        except OSError:
            continue
        for sym in ("_ZN4absl12lts_2026010713hash_internal10CityHash64EPKcm",):
            f = getattr(lib, sym, None)
            if f is not None:
                f.restype = ctypes.c_uint64
                f.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
                return f
    pytest.skip("no absl CityHash64 export found")


def test_farmhash_na_0to32_matches_independent_cityhash64(orc):
    # farmhashna::Hash64 for len <= 32 is CityHash64 v1.1 (HashLen0to16,
    # HashLen17to32: same constants k0/k1/k2, Rotate(b,37)/Rotate(a,25),
    # HashLen16 with mul).  The 8-16 B branch is the C3 key path (farm_16 on
    # the GPU, rsk_device.h); 33-64 B is where the two functions diverge.
    city = _absl_cityhash64()
    rng = np.random.default_rng(7)
    for n in range(0, 33):
        for _ in range(40):
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert orc.farmhash_na64(b) == city(b, n), n
            assert orc.farmhash_uo64(b) == city(b, n), n  # farmUo == na up to 64 B
    # and the 16-byte C3 stream keys themselves
    keys = orc.gen_keys16(0x5EED0003, 0, 2000).reshape(-1, 16)
    for i in range(2000):
        kb = keys[i].tobytes()
        assert orc.farmhash_uo64(kb) == city(kb, 16)
    b = rng.integers(0, 256, 40, dtype=np.uint8).tobytes()
    assert orc.farmhash_na64(b) != city(b, 40)  # the functions really differ above 32 B


@pytest.mark.parametrize("n,branch", [(3, "linear"), (20_000, "linear"), (45_000, "bias"), (50_000, "bias"),
                                      (65_000, "bias"), (200_000, "raw"), (3_000_000, "raw")])
def test_hll_estimator_branches_independent_restatement(orc, n, branch):
    # Pins the oracle's estimator (and through the golden vectors the GPU's) in
    # all three hllCount branches against a restatement that shares no code with
    # it; the bias-polynomial branch (2.5m <= E < 72000) is not reached by the
    # reference's own JUnit cases.  No Redis-produced value is available here
    # (no redis-server): against the Redis binary itself this stays unpinned.
    regs = np.zeros(orc.REGISTERS, np.uint8)
    orc.hll_add_gen16(regs, 0x5EED0002, 0, n)
    want, got_branch = redis32_hllcount_raw(regs)
    assert got_branch == branch
    assert orc.hll_count_raw(regs) == want


def test_zipf_stream_shape_and_subset_oracle(orc):
    # the Zipf(1.1) table: monotone, ends at 2^63, rank frequencies follow r^-1.1
    G, s = 10_000, 1.1
    cdf = orc.zipf_cdf(G, s)
    assert (np.diff(cdf.astype(np.float64)) >= 0).all() and int(cdf[-1]) == 1 << 63
    w = np.arange(1, G + 1, dtype=np.float64) ** -s
    assert abs(int(cdf[0]) / 2.0 ** 63 - w[0] / w.sum()) < 1e-12
    n = 400_000
    groups, keys = orc.gen_grouped_zipf(0x5EED0006, G, s, 0, n)
    freq = np.bincount(groups, minlength=G) / n
    assert abs(freq[0] - w[0] / w.sum()) < 0.01 and abs(freq[9] - w[9] / w.sum()) < 0.005
    # the pair-parallel subset oracle equals a direct replay of the stream
    gs = 64
    ref = np.zeros(gs * orc.REGISTERS, np.uint8)
    for j in np.nonzero(groups < gs)[0]:
        idx, c = orc.patlen(keys[16 * j:16 * j + 16].tobytes())
        o = int(groups[j]) * orc.REGISTERS + idx
        ref[o] = max(ref[o], c)
    for threads in (1, 3):
        sub = np.zeros(gs * orc.REGISTERS, np.uint8)
        orc.hll_add_gen_grouped_zipf_subset(sub, G, gs, s, 0x5EED0006, 0, n, threads)
        assert np.array_equal(sub, ref), threads


def test_full_pool_oracle_forms_match_the_sequential_ones(orc):
    """The multi-threaded full-pool oracle forms used by the every-sketch C5
    checks (groups generated alone, then each thread hashing the pairs of its
    own range of groups) give the same pools as the sequential generators."""
    G, n = 97, 40_000
    for zipf in (0.0, 1.1):
        if zipf:
            g_ref, k_ref = orc.gen_grouped_zipf(0x5EED0006, G, zipf, 123, n)
            groups = orc.gen_grouped_zipf_groups(0x5EED0006, G, zipf, 123, n, 4)
        else:
            g_ref, k_ref = orc.gen_grouped(0x5EED0006, G, 123, n)
            groups = orc.gen_grouped_groups(0x5EED0006, G, 123, n, 4)
        assert np.array_equal(groups, g_ref)
        ref = np.zeros((G, orc.REGISTERS), np.uint8)
        for gid in np.unique(g_ref):
            sel = g_ref == gid
            orc.hll_add(ref[gid], k_ref.reshape(-1, 16)[sel].reshape(-1), None, 16, int(sel.sum()))
        full = np.zeros((G, orc.REGISTERS), np.uint8)
        orc.hll_add_keys_by_groups(full, G, groups, 0x5EED0006, 123, 4)
        assert np.array_equal(full, ref), zipf
