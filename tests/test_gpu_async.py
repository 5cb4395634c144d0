"""The asynchronous C ABI (rsk_*_async, include/rsketch.h) -- the C side of
RHyperLogLogAsync / RBloomFilter futures (RHyperLogLogAsync.java:22-33;
CommandAsyncService.java:86-105): every accepted call fires its callback once
with the reply the synchronous call gives, calls on different handles may be
issued from several threads at once, host inputs may be reused as soon as the
call returns.  Also: rsk_trim, the now-synchronous rsk_hll_merge_batch, and the
Redis GET of an imported (SET) string returned byte-identical until the key is
next written."""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class Waiter:
    """Collects (status, value) of callbacks; keeps the ctypes thunk alive."""

    def __init__(self, lib):
        self.results = {}
        self.cond = threading.Condition()
        self.threads = set()

        def fire(user, status, value):
            user = user or 0  # ctypes hands a NULL void * over as None
            with self.cond:
                self.results[user] = (status, value)
                self.threads.add(threading.get_ident())
                self.cond.notify_all()

        self.fn = lib.DONE_FN(fire)

    def wait(self, keys, timeout=60):
        with self.cond:
            ok = self.cond.wait_for(lambda: all(k in self.results for k in keys), timeout)
        assert ok, "callbacks did not fire: %s" % [k for k in keys if k not in self.results]
        return [self.results[k] for k in keys]


@pytest.fixture(scope="module")
def L():
    from redisson_amd import _lib

    return _lib.load()


def _pool(L, engine, n=1):
    from redisson_amd import _lib

    h = ctypes.c_void_p()
    _lib.check(L.rsk_hll_create(engine.ctx, n, ctypes.byref(h)))
    return h


def test_hll_async_matches_sync(L, engine, orc):
    from redisson_amd import KeyBatch, _lib, devmem

    w = Waiter(_lib)
    h = _pool(L, engine, 4)
    keys = orc.gen_keys16(0x5EED0002, 0, 300_000)
    ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
    _lib.check(L.rsk_hll_add_async(h, 0, ctypes.byref(ks), w.fn, 1))
    keys[:] = 0  # host input reusable at once: the call staged its own copy
    _lib.check(L.rsk_hll_add_async(h, 0, ctypes.byref(ks), w.fn, 2))  # all-zero keys: one more register at most
    (s1, v1), (s2, v2) = w.wait([1, 2])
    assert s1 == s2 == 0 and v1 == 1
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, orc.gen_keys16(0x5EED0002, 0, 300_000), None, 16, 300_000)
    orc.hll_add(ref, keys, None, 16, 300_000)
    out = np.zeros(16384, np.uint8)
    _lib.check(L.rsk_hll_get_registers(h, 0, out.ctypes.data, _lib.RSK_MEM_HOST))
    assert np.array_equal(out, ref)
    # a repeat changes nothing: reply 0 (device-resident keys)
    dk = devmem.gen_keys16(engine, 0x5EED0002, 0, 300_000)
    kd = dk.keys_fixed(300_000, 16).as_struct()
    _lib.check(L.rsk_hll_add_async(h, 0, ctypes.byref(kd), w.fn, 3))
    assert w.wait([3]) == [(0, 0)]
    # PFCOUNT, countWith, mergeWith, batched mergeWith
    _lib.check(L.rsk_hll_add_async(h, 1, ctypes.byref(kd), w.fn, 4))
    _lib.check(L.rsk_hll_count_async(h, 0, w.fn, 5))
    hs = (ctypes.c_void_p * 2)(h.value, h.value)
    ids = (ctypes.c_uint64 * 2)(0, 3)  # 3 does not exist: skipped like a missing key
    _lib.check(L.rsk_hll_count_union_async(hs, ids, 2, w.fn, 6))
    src = (ctypes.c_void_p * 1)(h.value)
    sid = (ctypes.c_uint64 * 1)(1)
    _lib.check(L.rsk_hll_merge_async(h, 2, src, sid, 1, w.fn, 7))
    d_ids = np.array([3], np.uint64)
    s_ids = np.array([2], np.uint64)
    _lib.check(L.rsk_hll_merge_batch_async(h, d_ids.ctypes.data, s_ids.ctypes.data, 1, w.fn, 8))
    res = w.wait([4, 5, 6, 7, 8])
    assert res[0] == (0, 1)
    assert res[1] == (0, orc.hll_count_dense(ref))
    assert res[2] == (0, orc.hll_count_raw(ref))
    assert res[3][0] == 0 and res[4][0] == 0
    sync = np.zeros(4, np.uint64)
    _lib.check(L.rsk_hll_count(h, None, 4, sync.ctypes.data))
    ref1 = np.zeros(16384, np.uint8)
    orc.hll_add(ref1, dk.to_numpy(), None, 16, 300_000)
    assert int(sync[2]) == int(sync[3]) == orc.hll_count_dense(ref1)
    dk.free()
    L.rsk_hll_destroy(h)


def test_two_handles_concurrently(L, engine, orc):
    """Two threads, two handles, async adds issued at once: both callbacks
    fire with the right replies and both sketches hold their own keys."""
    from redisson_amd import KeyBatch, _lib

    w = Waiter(_lib)
    hs = [_pool(L, engine) for _ in range(2)]
    batches = [orc.gen_keys16(0x5EED0100 + t, 0, 200_000) for t in range(2)]
    go = threading.Barrier(2)
    errs = []

    def issue(t):
        try:
            ks = KeyBatch.from_numpy(batches[t].reshape(-1, 16)).as_struct()
            go.wait()
            for r in range(4):  # the first creates the key (reply 1), repeats change nothing
                _lib.check(L.rsk_hll_add_async(hs[t], 0, ctypes.byref(ks), w.fn, 10 * t + r))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=issue, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs
    res = w.wait([0, 1, 2, 3, 10, 11, 12, 13])
    assert [v for _, v in res] == [1, 0, 0, 0, 1, 0, 0, 0]
    assert threading.get_ident() not in w.threads  # completed on the runtime's thread
    for t in range(2):
        ref = np.zeros(16384, np.uint8)
        orc.hll_add(ref, batches[t], None, 16, 200_000)
        out = np.zeros(16384, np.uint8)
        _lib.check(L.rsk_hll_get_registers(hs[t], 0, out.ctypes.data, _lib.RSK_MEM_HOST))
        assert np.array_equal(out, ref)
        L.rsk_hll_destroy(hs[t])


def test_bloom_async_replies_and_contains(L, engine, orc):
    from redisson_amd import KeyBatch, _lib

    w = Waiter(_lib)
    size, k, n = 958506, 7, 100_000
    b = ctypes.c_void_p()
    _lib.check(L.rsk_bloom_create(engine.ctx, size, k, ctypes.byref(b)))
    keys = orc.gen_keys16(0x5EED0003, 0, n)
    vk = [bytes(keys[16 * i: 16 * i + 16]) for i in range(n)] + [b"", b"x" * 70]
    batch = KeyBatch.from_bytes_list(vk)  # owns the blob and offsets the struct points at
    kb = batch.as_struct()
    added = np.full(len(vk), 7, np.uint8)
    _lib.check(L.rsk_bloom_add_async(b, ctypes.byref(kb), added.ctypes.data, w.fn, 1))
    got = np.zeros(len(vk), np.uint8)
    _lib.check(L.rsk_bloom_contains_async(b, ctypes.byref(kb), got.ctypes.data, w.fn, 2))
    assert w.wait([1, 2]) == [(0, len(vk)), (0, len(vk))]
    bits = np.zeros((size + 7) // 8, np.uint8)
    blob, offs = orc.pack_keys(vk)
    want = orc.bloom_add_batch(bits, size, k, blob, offs)
    assert np.array_equal(added, want)
    assert got.all()
    # reply-less add, device bits equal the oracle's
    _lib.check(L.rsk_bloom_add_async(b, ctypes.byref(kb), None, w.fn, 3))
    assert w.wait([3]) == [(0, len(vk))]
    out = np.zeros_like(bits)
    nb = ctypes.c_size_t()
    _lib.check(L.rsk_bloom_export_bits(b, out.ctypes.data, out.size, ctypes.byref(nb)))
    assert np.array_equal(out, bits)
    # refused calls never fire
    with pytest.raises(_lib.IllegalArgumentException):
        _lib.check(L.rsk_bloom_contains_async(b, ctypes.byref(kb), None, w.fn, 4))
    L.rsk_bloom_destroy(b)
    assert 4 not in w.results


def test_large_host_batch_completes_inline(L, engine, orc):
    """A host batch above 256 MiB is not pinned whole: it runs before the call
    returns and the callback fires on the calling thread."""
    from redisson_amd import KeyBatch, _lib

    w = Waiter(_lib)
    n = (256 << 20) // 16 + 1000
    keys = np.frombuffer(np.random.default_rng(3).bytes(16 * n), np.uint8)
    h = _pool(L, engine)
    ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
    _lib.check(L.rsk_hll_add_async(h, 0, ctypes.byref(ks), w.fn, 1))
    assert 1 in w.results and threading.get_ident() in w.threads
    assert w.results[1] == (0, 1)
    ref = np.zeros(16384, np.uint8)
    orc.hll_add_fixed_mt(ref, keys, 16, n, 8)
    out = np.zeros(16384, np.uint8)
    _lib.check(L.rsk_hll_get_registers(h, 0, out.ctypes.data, _lib.RSK_MEM_HOST))
    assert np.array_equal(out, ref)
    L.rsk_hll_destroy(h)


def test_trim_and_synchronous_merge_batch(L, engine, orc):
    from redisson_amd import KeyBatch, _lib

    h = _pool(L, engine, 3)
    keys = orc.gen_keys16(0x5EED0002, 0, 50_000)
    ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
    _lib.check(L.rsk_hll_add(h, 0, ctypes.byref(ks), None))
    d = np.array([1, 2], np.uint64)
    s = np.array([0, 1], np.uint64)  # 2 <- 1 <- 0: ordered by level
    _lib.check(L.rsk_hll_merge_batch(h, d.ctypes.data, s.ctypes.data, 2))
    # returns with the merges done: the registers read on any stream are final
    out = np.zeros(16384, np.uint8)
    _lib.check(L.rsk_hll_get_registers(h, 2, out.ctypes.data, _lib.RSK_MEM_HOST))
    ref = np.zeros(16384, np.uint8)
    orc.hll_add(ref, keys, None, 16, 50_000)
    assert np.array_equal(out, ref)
    _lib.check(L.rsk_trim(engine.ctx))
    cnt = np.zeros(3, np.uint64)
    _lib.check(L.rsk_hll_count(h, None, 3, cnt.ctypes.data))  # scratch regrown on demand
    assert len(set(cnt.tolist())) == 1
    L.rsk_hll_destroy(h)


def _sparse(ops):
    """A Redis sparse HLL string from (kind, value, run) opcodes."""
    out = bytearray(b"HYLL" + bytes([1, 0, 0, 0]) + bytes(8))
    for kind, v, run in ops:
        if kind == "zero":
            out.append(run - 1)
        elif kind == "xzero":
            out += bytes([0x40 | ((run - 1) >> 8), (run - 1) & 0xFF])
        else:
            out.append(0x80 | ((v - 1) << 2) | (run - 1))
    return bytes(out)


def test_import_returns_set_bytes_until_written(L, engine, orc):
    """SET of a non-canonical sparse string (VAL 3 x3 then VAL 3 x2, where the
    canonical form is x4 + x1) is what GET returns until the key is written;
    PFCOUNT only refreshes the card bytes; a PFADD re-encodes (registers
    unchanged by the import either way)."""
    from redisson_amd import KeyBatch, _lib

    s = _sparse([("val", 3, 3), ("val", 3, 2), ("xzero", 0, 16384 - 5)])
    h = _pool(L, engine)
    _lib.check(L.rsk_hll_import_redis(h, 0, s, len(s)))
    buf = (ctypes.c_uint8 * 12304)()
    n = ctypes.c_size_t()
    _lib.check(L.rsk_hll_export_redis(h, 0, buf, 12304, ctypes.byref(n)))
    assert bytes(buf[: n.value]) == s
    cnt = np.zeros(1, np.uint64)
    _lib.check(L.rsk_hll_count(h, None, 1, cnt.ctypes.data))
    _lib.check(L.rsk_hll_export_redis(h, 0, buf, 12304, ctypes.byref(n)))
    got = bytes(buf[: n.value])
    assert got[:8] == s[:8] and got[16:] == s[16:]
    assert int.from_bytes(got[8:16], "little") == int(cnt[0])  # the cached cardinality, valid
    keys = orc.gen_keys16(0x5EED0002, 0, 3)
    ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
    _lib.check(L.rsk_hll_add(h, 0, ctypes.byref(ks), None))
    _lib.check(L.rsk_hll_export_redis(h, 0, buf, 12304, ctypes.byref(n)))
    assert bytes(buf[16: n.value]) != s[16:]  # re-encoded after the write
    L.rsk_hll_destroy(h)


def test_grouped_pipeline_matches_sync(engine):
    """The pool's async forms (rsk_hll_add_grouped_async, rsk_hll_count_ids_async,
    rsk_hll_count_union_batch_async, rsk_hll_merge_batch_async), issued back to
    back, give what the synchronous calls give in the same order."""
    from redisson_amd import KeyBatch, devmem
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    G, n = 5000, 1 << 22
    groups, gkeys = devmem.gen_grouped(engine, 0x5EED0107, G, 0, n)
    kb = gkeys.keys_fixed(n, 16)
    rng = np.random.default_rng(3)
    cw = np.stack([rng.integers(0, G, 2000, dtype=np.uint64), rng.integers(0, G, 2000, dtype=np.uint64)], 1)
    md = rng.integers(0, G, 2000, dtype=np.uint64)
    ms = rng.integers(0, G, 2000, dtype=np.uint64)
    hkeys = np.frombuffer(rng.bytes(16 * 3000), np.uint8).reshape(3000, 16).copy()
    hg = rng.integers(0, G, 3000, dtype=np.uint32)
    ref, got = GroupedHyperLogLog(engine, G), GroupedHyperLogLog(engine, G)
    try:
        ref.add(kb, groups)
        c_ref = ref.count().copy()
        w_ref = ref.countWith(cw)
        ref.mergeWith(md, ms)
        ref.add(KeyBatch.from_numpy(hkeys), hg)
        c2_ref = ref.count().copy()
        for _ in range(2):  # twice: the second round starts from a cleared pool
            got.clear()
            c_out, w_out, c2_out = np.zeros(G, np.uint64), np.zeros(len(cw), np.uint64), np.zeros(G, np.uint64)
            hk = hkeys.copy()
            ops = [got.add_async(kb, groups), got.count_async(c_out), got.countWith_async(cw, w_out),
                   got.mergeWith_async(md, ms), got.add_async(KeyBatch.from_numpy(hk), hg), got.count_async(c2_out)]
            hk[:] = 0  # host keys were staged by the call
            assert ops[0].wait(60) == n
            for op in ops[1:]:
                op.wait(60)
            assert np.array_equal(c_out, c_ref)
            assert np.array_equal(w_out, w_ref)
            assert np.array_equal(c2_out, c2_ref)
        ids = np.array([7, 0, G - 1, 7], np.uint64)
        sub = np.zeros(4, np.uint64)
        got.count_async(sub, ids).wait(60)
        assert np.array_equal(sub, c2_ref[ids.astype(np.int64)])
    finally:
        ref.close()
        got.close()


def test_callbacks_ordered_and_off_the_stream(L, engine):
    """Callbacks fire in submission order on the context's completion thread;
    a callback that blocks does not hold up later device work (a synchronous
    call issued behind it returns while it is still blocked), and rsk_sync
    returns only after every earlier callback has returned."""
    from redisson_amd import _lib

    h = _pool(L, engine, 2)
    release = threading.Event()
    order, released = [], []

    def fire(user, status, value):
        user = user or 0
        if user == 1:
            released.append(release.wait(20))
        order.append((user, status))

    fn = _lib.DONE_FN(fire)
    try:
        for u in range(1, 21):
            _lib.check(L.rsk_hll_count_async(h, u % 2, fn, u))
        out = np.zeros(2, np.uint64)
        _lib.check(L.rsk_hll_count(h, None, 2, out.ctypes.data))  # behind 20 queued completions
        assert out.tolist() == [0, 0]
        release.set()
        _lib.check(L.rsk_sync(engine.ctx))
        assert released == [True], "the synchronous call waited for a blocked callback"
        assert order == [(u, 0) for u in range(1, 21)]
    finally:
        release.set()
        L.rsk_sync(engine.ctx)
        L.rsk_hll_destroy(h)


def test_async_reads_back_state_at_call_time(engine):
    """Read-backs run on the output copy stream and staged inputs on the
    input stream: an async count still answers with the pool as it stood at
    its call, when a synchronous add to the same pool follows at once, and an
    async add of host keys whose buffer is overwritten after the call adds
    the keys as they were."""
    from redisson_amd import KeyBatch
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    G = 3000
    rng = np.random.default_rng(11)
    ka = np.frombuffer(rng.bytes(16 * 200_000), np.uint8).reshape(-1, 16).copy()
    ga = rng.integers(0, G, len(ka), dtype=np.uint32)
    kb = np.frombuffer(rng.bytes(16 * 150_000), np.uint8).reshape(-1, 16).copy()
    gb = rng.integers(0, G, len(kb), dtype=np.uint32)
    ref, got = GroupedHyperLogLog(engine, G), GroupedHyperLogLog(engine, G)
    try:
        ref.add(KeyBatch.from_numpy(ka), ga)
        c_a = ref.count().copy()
        ref.add(KeyBatch.from_numpy(kb), gb)
        c_ab = ref.count().copy()
        for _ in range(3):
            got.clear()
            got.add(KeyBatch.from_numpy(ka), ga)
            out1, out2 = np.zeros(G, np.uint64), np.zeros(G, np.uint64)
            op1 = got.count_async(out1)
            got.add(KeyBatch.from_numpy(kb), gb)  # synchronous, right behind the async count
            op2 = got.count_async(out2)
            op1.wait(60)
            op2.wait(60)
            assert np.array_equal(out1, c_a)
            assert np.array_equal(out2, c_ab)
            got.clear()
            hk = ka.copy()
            op3 = got.add_async(KeyBatch.from_numpy(hk), ga)
            hk[:] = 0  # the call staged its own copy
            out3 = np.zeros(G, np.uint64)
            op4 = got.count_async(out3)
            op3.wait(60)
            op4.wait(60)
            assert np.array_equal(out3, c_a)
    finally:
        ref.close()
        got.close()


def _noncanonical(canon: bytes) -> bytes:
    """The same registers as a canonical sparse string, re-encoded with its first
    long zero run (XZERO of 130+) cut into XZERO + ZERO 64: two zero opcodes in
    a row, which the canonical encoder never writes."""
    body, out, i = canon[16:], bytearray(), 0
    done = False
    while i < len(body):
        b = body[i]
        if (b & 0xC0) == 0x40:
            run = (((b & 0x3F) << 8) | body[i + 1]) + 1
            if not done and run >= 130:
                r = run - 64
                out += bytes([0x40 | ((r - 1) >> 8), (r - 1) & 0xFF, 63])
                done = True
            else:
                out += body[i:i + 2]
            i += 2
        else:
            out.append(b)
            i += 1
    assert done
    return canon[:16] + bytes(out)


def test_async_add_keeps_set_string_when_nothing_changes(L, engine, orc):
    """a PFADD that changes no register leaves a kept SET string in
    place -- rsk_hll_add, rsk_hll_add_async and rsk_hll_add_each (host replies)
    alike; one that changes a register re-encodes it (async too)."""
    from redisson_amd import KeyBatch, _lib

    keys = orc.gen_keys16(0x5EED0002, 0, 40)
    regs = np.zeros(16384, np.uint8)
    orc.hll_add(regs, keys, None, 16, 40)
    s = _noncanonical(orc.hll_encode_sparse(regs))
    h = _pool(L, engine)
    ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
    buf = (ctypes.c_uint8 * 12304)()
    n = ctypes.c_size_t()

    def get():
        _lib.check(L.rsk_hll_export_redis(h, 0, buf, 12304, ctypes.byref(n)))
        return bytes(buf[: n.value])

    b = (ctypes.c_uint8 * len(s)).from_buffer_copy(s)
    _lib.check(L.rsk_hll_import_redis(h, 0, b, len(s)))
    assert get() == s
    op = _lib.NativeOp(ks)
    op.issued(L.rsk_hll_add_async(h, 0, ctypes.byref(ks), op.fn, None))
    assert op.wait(30) == 0 and get() == s  # nothing changed: still the SET bytes
    ch = ctypes.c_uint8()
    _lib.check(L.rsk_hll_add(h, 0, ctypes.byref(ks), ctypes.byref(ch)))
    assert ch.value == 0 and get() == s
    out = np.zeros(40, np.uint8)
    _lib.check(L.rsk_hll_add_each(h, 0, ctypes.byref(ks), out.ctypes.data))
    assert not out.any() and get() == s
    more = orc.gen_keys16(0x5EED0002, 1000, 50)
    km = KeyBatch.from_numpy(more.reshape(-1, 16)).as_struct()
    op = _lib.NativeOp(km)
    op.issued(L.rsk_hll_add_async(h, 0, ctypes.byref(km), op.fn, None))
    assert op.wait(30) == 1
    orc.hll_add(regs, more, None, 16, 50)
    assert get()[16:] == orc.hll_encode_sparse(regs)[16:]  # re-encoded canonically
    L.rsk_hll_destroy(h)
