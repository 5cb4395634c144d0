"""The reference's own JUnit tests, replayed through the redisson_amd mirror of
the Java API on the GPU (T/RedissonHyperLogLogTest.java, T/RedissonBloomFilterTest.java)."""
import numpy as np
import pytest

from redisson_amd import IllegalArgumentException, IllegalStateException

pytestmark = pytest.mark.gpu


def test_hll_testAdd(client):
    log = client.getHyperLogLog("log")
    log.add(1)
    log.add(2)
    log.add(3)
    assert log.count() == 3


def test_hll_testMerge(client):
    hll1 = client.getHyperLogLog("hll1")
    assert hll1.add("foo")
    assert hll1.add("bar")
    assert hll1.add("zap")
    assert hll1.add("a")
    hll2 = client.getHyperLogLog("hll2")
    assert hll2.add("a")
    assert hll2.add("b")
    assert hll2.add("c")
    assert hll2.add("foo")
    assert not hll2.add("c")
    hll3 = client.getHyperLogLog("hll3")
    hll3.mergeWith("hll1", "hll2")
    assert hll3.count() == 6


def test_hll_countWith_and_missing_keys(client, orc):
    a = client.getHyperLogLog("a")
    b = client.getHyperLogLog("b")
    assert a.count() == 0
    a.addAll(["x%d" % i for i in range(1000)])
    b.addAll(["x%d" % i for i in range(500, 1500)])
    r = orc.RedisModel()
    r.pfadd("a", *[('"x%d"' % i).encode() for i in range(1000)])
    r.pfadd("b", *[('"x%d"' % i).encode() for i in range(500, 1500)])
    assert a.countWith("b") == r.pfcount("a", "b")
    assert a.countWith("b", "nosuchkey") == r.pfcount("a", "b", "nosuchkey")
    assert a.count() == r.pfcount("a")
    assert a.addAll([]) is False  # existing key, nothing added
    assert client.getHyperLogLog("fresh").addAll([]) is True  # key created


def test_hll_batch_pipelined_adds(client, orc):
    batch = client.createBatch()
    h = batch.getHyperLogLog("pipe")
    futs = [h.addAsync(i % 700) for i in range(2000)]
    res = batch.execute()
    r = orc.RedisModel()
    want = [bool(r.pfadd("pipe", str(i % 700).encode())) for i in range(2000)]
    assert res == want and [f.result() for f in futs] == want
    assert client.getHyperLogLog("pipe").count() == r.pfcount("pipe")


def test_bitset_batch_pipelined_commands(client, orc):
    # RBatch.getBitSet (RedissonBatch.java:191): SETBIT/GETBIT runs collapse into
    # one launch each; every reply equals the in-order Redis model's.
    batch = client.createBatch()
    b = batch.getBitSet("bbits")
    rng = np.random.default_rng(11)
    offs = rng.integers(0, 5000, 300).tolist()
    r = orc.RedisModel()
    futs, want = [], []
    for t, o in enumerate(offs):
        if t % 7 == 3:
            futs.append(b.clearAsync(o))
            r.setbit("bbits", o, 0)
            want.append(None)
        elif t % 5 == 4:
            futs.append(b.getAsync(o))
            want.append(bool(r.getbit("bbits", o)))
        else:
            futs.append(b.setAsync(o))
            r.setbit("bbits", o, 1)
            want.append(None)
    futs.append(b.cardinalityAsync())
    want.append(r.bitcount("bbits"))
    futs.append(b.setAsync(100, 200))
    for o in range(100, 200):
        r.setbit("bbits", o, 1)
    want.append(None)
    futs.append(b.clearAsync(150, 160))
    for o in range(150, 160):
        r.setbit("bbits", o, 0)
    want.append(None)
    futs.append(b.lengthAsync())
    futs.append(b.toByteArrayAsync())
    futs.append(b.getAsync(155))
    res = batch.execute()
    raw = r.get("bbits")
    length = max((i for i in range(8 * len(raw)) if raw[i >> 3] & (0x80 >> (i & 7))), default=-1) + 1
    want += [length, raw, False]
    assert res == want and [f.result() for f in futs] == want


def test_hll_redis_roundtrip(client, orc):
    h = client.getHyperLogLog("rt")
    h.addAll(list(range(5000)))
    s = h.toRedisBytes()
    g = client.getHyperLogLog("rt2")
    g.fromRedisBytes(s)
    assert np.array_equal(g.registers(), h.registers())
    assert g.count() == h.count()


def test_bloom_testConfig(client):
    f = client.getBloomFilter("filter")
    f.tryInit(100, 0.03)
    assert f.getExpectedInsertions() == 100
    assert f.getFalseProbability() == 0.03
    assert f.getHashIterations() == 5
    assert f.getSize() == 729


def test_bloom_testInit(client):
    f = client.getBloomFilter("filter")
    assert f.tryInit(55000000, 0.03)
    assert not f.tryInit(55000001, 0.03)
    f.delete()
    assert f.tryInit(55000001, 0.03)


def test_bloom_not_initialized(client):
    f = client.getBloomFilter("filter")
    with pytest.raises(IllegalStateException):
        f.getExpectedInsertions()
    with pytest.raises(IllegalStateException):
        f.contains("32")
    with pytest.raises(IllegalStateException):
        f.add("123")


def test_bloom_test(client):
    f = client.getBloomFilter("filter")
    f.tryInit(550000000, 0.03)
    assert not f.contains("123")
    assert f.add("123")
    assert f.contains("123")
    assert not f.add("123")
    assert f.count() == 1
    assert not f.contains("hflgs;jl;ao1-32471320o31803-24")
    assert f.add("hflgs;jl;ao1-32471320o31803-24")
    assert f.contains("hflgs;jl;ao1-32471320o31803-24")
    assert f.count() == 2


def test_bloom_max_size(client):
    f = client.getBloomFilter("big")
    with pytest.raises(IllegalArgumentException):
        f.tryInit(10 ** 9, 0.01)
