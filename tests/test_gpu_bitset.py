"""RBitSet on the GPU: the reference's JUnit tests (T/RedissonBitSetTest.java)
replayed through the mirror, plus batched SETBIT/GETBIT/BITOP/BITCOUNT parity
against the oracle's Redis model."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_testIndexRange(client):
    bs = client.getBitSet("testbitset")
    top = 2147483647 * 2
    assert not bs.get(top)
    bs.set(top)
    assert bs.get(top)


def test_testLength(client):
    bs = client.getBitSet("testbitset")
    bs.set(0, 5)
    bs.clear(0, 1)
    assert bs.length() == 5
    bs.clear()
    bs.set(28)
    bs.set(31)
    assert bs.length() == 32
    bs.clear()
    bs.set(3)
    bs.set(7)
    assert bs.length() == 8
    bs.clear()
    bs.set(3)
    bs.set(120)
    bs.set(121)
    assert bs.length() == 122
    bs.clear()
    bs.set(0)
    assert bs.length() == 1


def test_testClear(client):
    bs = client.getBitSet("testbitset")
    bs.set(0, 8)
    bs.clear(0, 3)
    assert bs.toString() == "{3, 4, 5, 6, 7}"


def test_testNot(client):
    bs = client.getBitSet("testbitset")
    bs.set(3)
    bs.set(5)
    getattr(bs, "not")()
    assert bs.toString() == "{0, 1, 2, 4, 6, 7}"


def test_testSet(client):
    from redisson_amd.bitset import JavaBitSet

    bs = client.getBitSet("testbitset")
    bs.set(3)
    bs.set(5)
    assert bs.toString() == "{3, 5}"
    bs1 = JavaBitSet()
    bs1.set(1)
    bs1.set(10)
    bs.set(bs1)
    bs = client.getBitSet("testbitset")
    assert bs.toString() == "{1, 10}"


def test_testSetGet(client):
    bitset = client.getBitSet("testbitset")
    assert bitset.cardinality() == 0
    assert bitset.size() == 0
    bitset.set(10, True)
    bitset.set(31, True)
    assert not bitset.get(0)
    assert bitset.get(31)
    assert bitset.get(10)
    assert bitset.cardinality() == 2
    assert bitset.size() == 32


def test_testSetRange(client):
    bs = client.getBitSet("testbitset")
    bs.set(3, 10)
    assert bs.cardinality() == 7
    assert bs.size() == 16


def test_testAsBitSet(client):
    bs = client.getBitSet("testbitset")
    bs.set(3, True)
    bs.set(41, True)
    assert bs.size() == 48
    bitset = bs.asBitSet()
    assert bitset.get(3)
    assert bitset.get(41)
    assert bs.cardinality() == 2


def test_testAnd(client):
    bs1 = client.getBitSet("testbitset1")
    bs1.set(3, 5)
    assert bs1.cardinality() == 2
    assert bs1.size() == 8
    bs2 = client.getBitSet("testbitset2")
    bs2.set(4)
    bs2.set(10)
    getattr(bs1, "and")(bs2.getName())
    assert not bs1.get(3)
    assert bs1.get(4)
    assert not bs1.get(5)
    assert bs2.get(10)
    assert bs1.cardinality() == 1
    assert bs1.size() == 16


def test_batched_bitops_match_redis_model(client, orc):
    rng = np.random.default_rng(9)
    r = orc.RedisModel()
    names = ["a", "b", "c"]
    for nm in names:
        idx = rng.integers(0, 200000, 5000)
        client.getBitSet(nm).setBits(idx.tolist())
        for i in idx:
            r.setbit(nm, int(i), 1)
        clr = rng.integers(0, 250000, 500)
        client.getBitSet(nm).setBits(clr.tolist(), False)
        for i in clr:
            r.setbit(nm, int(i), 0)
    for nm in names:
        bs = client.getBitSet(nm)
        assert bs.toByteArray() == r.get(nm)
        assert bs.cardinality() == r.bitcount(nm)
        assert bs.size() == 8 * r.strlen(nm)
        q = rng.integers(0, 300000, 3000)
        assert bs.getBits(q) == [bool(r.getbit(nm, int(i))) for i in q]
    getattr(client.getBitSet("a"), "or")("b", "c")
    r.bitop("OR", "a", "a", "b", "c")
    assert client.getBitSet("a").toByteArray() == r.get("a")
    client.getBitSet("b").xor("c", "missing")
    r.bitop("XOR", "b", "b", "c", "missing")
    assert client.getBitSet("b").toByteArray() == r.get("b")
    getattr(client.getBitSet("c"), "not")()
    r.bitop("NOT", "c", "c")
    assert client.getBitSet("c").toByteArray() == r.get("c")
