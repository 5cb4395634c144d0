"""The reference's reactive JUnit tests replayed through the reactive mirror
(T/RedissonHyperLogLogReactiveTest.java, T/RedissonBitSetReactiveTest.java);
sync() is Publisher.block(), as BaseReactiveTest.sync (T/BaseReactiveTest.java:76)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture()
def redisson():
    from redisson_amd import Redisson

    r = Redisson.createReactive()
    yield r
    r.shutdown()


def sync(p):
    return p.block()


def test_hll_testAdd(redisson):
    log = redisson.getHyperLogLog("log")
    sync(log.add(1))
    sync(log.add(2))
    sync(log.add(3))
    assert sync(log.count()) == 3


def test_hll_testMerge(redisson):
    hll1 = redisson.getHyperLogLog("hll1")
    assert sync(hll1.add("foo"))
    assert sync(hll1.add("bar"))
    assert sync(hll1.add("zap"))
    assert sync(hll1.add("a"))
    hll2 = redisson.getHyperLogLog("hll2")
    assert sync(hll2.add("a"))
    assert sync(hll2.add("b"))
    assert sync(hll2.add("c"))
    assert sync(hll2.add("foo"))
    assert not sync(hll2.add("c"))
    hll3 = redisson.getHyperLogLog("hll3")
    assert sync(hll3.mergeWith("hll1", "hll2")) is None
    assert sync(hll3.count()) == 6


def test_publisher_is_cold_and_signals(redisson):
    log = redisson.getHyperLogLog("cold")
    p = log.addAll(["x%d" % i for i in range(100)])
    assert sync(log.count()) == 0  # nothing ran before a subscription
    seen, done = [], []
    p.subscribe(on_next=seen.append, on_complete=lambda: done.append(1)).result()
    assert seen == [True] and done == [1]
    assert sync(log.count()) == sync(redisson.getHyperLogLog("cold").count()) > 90
    sync(redisson.getBitSet("not-an-hll").set(1))
    errs = []
    redisson.getHyperLogLog("cold").countWith("not-an-hll").subscribe(on_error=errs.append).result()
    from redisson_amd import RedisException

    assert len(errs) == 1 and isinstance(errs[0], RedisException)  # WRONGTYPE, as Redis replies


def test_bitset_testLength(redisson):
    bs = redisson.getBitSet("testbitset")
    sync(bs.set(0, 5))
    sync(bs.clear(0, 1))
    assert sync(bs.length()) == 5
    sync(bs.clear())
    sync(bs.set(28))
    sync(bs.set(31))
    assert sync(bs.length()) == 32
    sync(bs.clear())
    sync(bs.set(3))
    sync(bs.set(7))
    assert sync(bs.length()) == 8
    sync(bs.clear())
    sync(bs.set(3))
    sync(bs.set(120))
    sync(bs.set(121))
    assert sync(bs.length()) == 122
    sync(bs.clear())
    sync(bs.set(0))
    assert sync(bs.length()) == 1


def test_bitset_testClear(redisson):
    bs = redisson.getBitSet("testbitset")
    sync(bs.set(0, 8))
    sync(bs.clear(0, 3))
    assert bs.toString() == "{3, 4, 5, 6, 7}"


def test_bitset_testNot(redisson):
    bs = redisson.getBitSet("testbitset")
    sync(bs.set(3))
    sync(bs.set(5))
    sync(getattr(bs, "not")())
    assert bs.toString() == "{0, 1, 2, 4, 6, 7}"


def test_bitset_testSet(redisson):
    from redisson_amd.bitset import JavaBitSet

    bs = redisson.getBitSet("testbitset")
    sync(bs.set(3))
    sync(bs.set(5))
    assert bs.toString() == "{3, 5}"
    sync(bs.set(JavaBitSet([1, 10])))
    bs = redisson.getBitSet("testbitset")
    assert bs.toString() == "{1, 10}"


def test_bitset_testSetGet(redisson):
    bitset = redisson.getBitSet("testbitset")
    assert sync(bitset.cardinality()) == 0
    assert sync(bitset.size()) == 0
    sync(bitset.set(10, True))
    sync(bitset.set(31, True))
    assert not sync(bitset.get(0))
    assert sync(bitset.get(31))
    assert sync(bitset.get(10))
    assert sync(bitset.cardinality()) == 2
    assert sync(bitset.size()) == 32


def test_bitset_testSetRange(redisson):
    bs = redisson.getBitSet("testbitset")
    sync(bs.set(3, 10))
    assert sync(bs.cardinality()) == 7
    assert sync(bs.size()) == 16


def test_bitset_testAsBitSet(redisson):
    bs = redisson.getBitSet("testbitset")
    sync(bs.set(3, True))
    sync(bs.set(41, True))
    assert sync(bs.size()) == 48
    bitset = sync(bs.asBitSet())
    assert bitset.get(3) and bitset.get(41)
    assert bitset.cardinality() == 2


def test_bitset_testAnd(redisson):
    bs1 = redisson.getBitSet("testbitset1")
    sync(bs1.set(3, 5))
    assert sync(bs1.cardinality()) == 2
    assert sync(bs1.size()) == 8
    bs2 = redisson.getBitSet("testbitset2")
    sync(bs2.set(4))
    sync(bs2.set(10))
    sync(getattr(bs1, "and")(bs2.getName()))
    assert not sync(bs1.get(3))
    assert sync(bs1.get(4))
    assert not sync(bs1.get(5))
    assert sync(bs2.get(10))
    assert sync(bs1.cardinality()) == 1
    assert sync(bs1.size()) == 16
