"""RBitSet on the GPU: the reference's JUnit tests (T/RedissonBitSetTest.java)
replayed through the mirror, plus batched SETBIT/GETBIT/BITOP/BITCOUNT parity
against the oracle's Redis model."""
import ctypes
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


def _bs(L, engine, data: bytes):
    import ctypes

    from redisson_amd import _lib

    b = ctypes.c_void_p()
    _lib.check(L.rsk_bitset_create(engine.ctx, ctypes.byref(b)))
    arr = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    _lib.check(L.rsk_bitset_set_bytes(b, arr.ctypes.data, len(data)))
    return b


def _bytes(L, b) -> bytes:
    import ctypes

    from redisson_amd import _lib

    n = ctypes.c_uint64()
    _lib.check(L.rsk_bitset_strlen(b, ctypes.byref(n)))
    out = np.zeros(max(1, n.value), np.uint8)
    ln = ctypes.c_size_t()
    _lib.check(L.rsk_bitset_get_bytes(b, out.ctypes.data, out.size, ctypes.byref(ln)))
    return out[: ln.value].tobytes()


def test_vectorized_bitop_length_range_edges(engine):
    """16-byte-chunk BITOP / length / set-range at lengths around the chunk
    size (Redis semantics: shorter sources zero-padded, NOT keeps no bits past
    the string, length = highest MSB-first set bit + 1)."""
    import ctypes
    import functools

    from redisson_amd import _lib

    L = _lib.load()
    rng = np.random.default_rng(21)
    for lens in [(1,), (15, 16, 17), (100003, 7, 4096), (31, 33), (64, 64)]:
        srcs = [rng.integers(0, 256, ln, dtype=np.uint8).tobytes() for ln in lens]
        mx = max(lens)
        pads = [np.frombuffer(x + b"\0" * (mx - len(x)), np.uint8) for x in srcs]
        for op, fn in ((0, np.bitwise_and), (1, np.bitwise_or), (2, np.bitwise_xor)):
            hs = [_bs(L, engine, x) for x in srcs]
            dst = _bs(L, engine, b"")
            arr = (ctypes.c_void_p * len(hs))(*[h.value for h in hs])
            _lib.check(L.rsk_bitset_bitop(op, dst, arr, len(hs)))
            assert _bytes(L, dst) == functools.reduce(fn, pads).tobytes(), (lens, op)
        h = _bs(L, engine, srcs[0])
        _lib.check(L.rsk_bitset_bitop(3, h, (ctypes.c_void_p * 1)(h.value), 1))  # NOT in place
        want = (~np.frombuffer(srcs[0], np.uint8)).astype(np.uint8)
        assert _bytes(L, h) == want.tobytes()
        cnt = ctypes.c_uint64()
        _lib.check(L.rsk_bitset_bitcount(h, ctypes.byref(cnt)))
        assert cnt.value == int(np.unpackbits(want).sum())  # no bits past the string
        z = _bs(L, engine, b"\0" * (len(srcs[0]) + 40))
        _lib.check(L.rsk_bitset_bitop(1, z, (ctypes.c_void_p * 2)(z.value, h.value), 2))
        assert _bytes(L, z) == want.tobytes() + b"\0" * 40
    # length(): sparse strings, the top bit anywhere in a chunk
    for n in (1, 16, 17, 1000, 65537):
        for _ in range(3):
            a = np.zeros(n, np.uint8)
            top = int(rng.integers(0, 8 * n))
            a[top >> 3] |= 0x80 >> (top & 7)
            low = rng.integers(0, top + 1, 5)
            for t in low:
                a[t >> 3] |= 0x80 >> (t & 7)
            h = _bs(L, engine, a.tobytes())
            out = ctypes.c_uint64()
            _lib.check(L.rsk_bitset_length(h, ctypes.byref(out)))
            assert out.value == top + 1
    # set_range([from, to), v) against the bit model, partial and whole bytes
    base = rng.integers(0, 256, 300, dtype=np.uint8)
    for frm, to, v in ((3, 5, 1), (3, 13, 1), (8, 16, 0), (5, 2000, 1), (0, 2400, 0), (17, 1601, 1), (9, 9, 1)):
        h = _bs(L, engine, base.tobytes())
        _lib.check(L.rsk_bitset_set_range(h, frm, to, v))
        bits = np.unpackbits(base)
        if to > frm:
            bits = np.concatenate([bits, np.zeros(max(0, to - bits.size), np.uint8)])
            bits[frm:to] = v
        assert _bytes(L, h) == np.packbits(bits).tobytes(), (frm, to, v)


def test_getBitSet_of_bloom_filter_is_its_bit_string(client, orc):
    """getBitSet(filterName) (Redisson.java:515-517) reads the bits
    RBloomFilter.add set: in Redis the filter's bits are the string key of that
    name.  GET / BITCOUNT / STRLEN / GETBIT equal the Redis model's after the
    reference's add() sequence (OracleBloomFilter replays
    RedissonBloomFilter.java:80-114 as SETBITs); writes through the RBitSet
    change what contains() sees; DEL of the string keeps the filter
    initialised with no bits."""
    from redisson_amd.codec import DEFAULT_CODEC

    r = orc.RedisModel()
    ref = orc.OracleBloomFilter(r, "bf", DEFAULT_CODEC.encode)
    bf = client.getBloomFilter("bf")
    assert bf.tryInit(300, 0.03) and ref.try_init(300, 0.03)
    bs = client.getBitSet("bf")
    assert bs.toByteArray() is None and bs.size() == 0 and bs.cardinality() == 0  # no SETBIT yet: no string
    elems = ["e%d" % i for i in range(200)]
    assert [bool(x) for x in bf.addAll(elems)] == [ref.add(e) for e in elems]
    assert bs.toByteArray() == r.get("bf")
    assert bs.cardinality() == r.bitcount("bf")
    assert bs.size() == 8 * r.strlen("bf")
    size = bf.getSize()
    q = list(range(0, size, 7))
    assert bs.getBits(q) == [bool(r.getbit("bf", i)) for i in q]
    assert bs.length() == max(i for i in range(size) if r.getbit("bf", i)) + 1
    # writes through the RBitSet: set a clear bit, clear a set one near the end
    clear_bits = [i for i in range(size) if not r.getbit("bf", i)]
    set_bits = [i for i in range(size) if r.getbit("bf", i)]
    bs.set(clear_bits[0])
    r.setbit("bf", clear_bits[0], 1)
    bs.clear(set_bits[-1])
    r.setbit("bf", set_bits[-1], 0)
    assert bs.toByteArray() == r.get("bf")  # STRLEN keeps the cleared byte, as Redis does
    assert bs.size() == 8 * r.strlen("bf")
    probe = elems + ["x%d" % i for i in range(200)]
    assert [bool(x) for x in bf.containsAll(probe)] == [ref.contains(e) for e in probe]
    assert bf.count() == ref.count()
    # DEL bf (RBitSet.delete): the string goes, {bf}__config stays
    assert bs.delete()
    r.delete("bf")
    assert bs.toByteArray() is None and bf.count() == 0
    assert bf.getHashIterations() == ref.k
    assert not any(bf.containsAll(elems))
    assert [bool(x) for x in bf.addAll(elems[:50])] == [ref.add(e) for e in elems[:50]]
    assert bs.toByteArray() == r.get("bf")
    # a SETBIT past the filter's string cannot be honoured on the GPU filter
    from redisson_amd import _lib

    with pytest.raises(_lib.IllegalArgumentException):
        bs.set((size + 7) // 8 * 8 + 100)


def test_bloom_view_rescans_only_after_writes(engine, orc):
    """the RBitSet view of a Bloom filter recomputes STRLEN (a scan of
    the whole filter) only when the filter was written since it last looked --
    GETBIT / GET / STRLEN repeated cost no scan -- and SET of the filter's
    string (rsk_bloom_import_bits) gives STRLEN = the SET length, trailing
    zero bytes included (Redis SET semantics), not a length left over from
    earlier writes through the view."""
    from redisson_amd import KeyBatch, _lib

    L = _lib.load()
    b = ctypes.c_void_p()
    _lib.check(L.rsk_bloom_create(engine.ctx, 1_000_003, 5, ctypes.byref(b)))
    v = ctypes.c_void_p()
    _lib.check(L.rsk_bloom_bitset(b, ctypes.byref(v)))

    def strlen():
        n = ctypes.c_uint64()
        _lib.check(L.rsk_bitset_strlen(v, ctypes.byref(n)))
        return n.value

    def scans():
        return engine.prof_read("bitset_length")[1]

    keys = orc.gen_keys16(0x5EED0003, 0, 2000)
    ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
    engine.prof_enable(True)
    engine.prof_reset()
    try:
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
        n0 = strlen()
        assert n0 > 0 and scans() == 1
        offs = np.arange(0, 1_000_000, 997, dtype=np.uint64)
        out = np.zeros(offs.size, np.uint8)
        for _ in range(5):
            _lib.check(L.rsk_bitset_getbits(v, offs.ctypes.data, offs.size, _lib.RSK_MEM_HOST, out.ctypes.data))
            assert strlen() == n0
        assert scans() == 1  # reads never rescan
        more = orc.gen_keys16(0x5EED0003, 2000, 2000)
        km = KeyBatch.from_numpy(more.reshape(-1, 16)).as_struct()
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(km), None))
        n1 = strlen()
        assert n1 >= n0 and scans() == 2  # one rescan after the write
        set_off = np.array([1_000_002], np.uint64)  # the filter's last bit
        _lib.check(L.rsk_bitset_setbits(v, set_off.ctypes.data, 1, 1, _lib.RSK_MEM_HOST))
        assert strlen() == 1_000_002 // 8 + 1 and scans() == 2  # the view's own write keeps its length
        s = bytes([0x80]) + bytes(99)  # SET of 100 bytes: bit 0 and 99 zero bytes
        buf = (ctypes.c_uint8 * len(s)).from_buffer_copy(s)
        _lib.check(L.rsk_bloom_import_bits(b, buf, len(s)))
        assert strlen() == 100
    finally:
        engine.prof_enable(False)
        L.rsk_bitset_destroy(v)
        L.rsk_bloom_destroy(b)
