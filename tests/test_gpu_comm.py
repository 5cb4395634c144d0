"""RCCL merge layer on one GPU (a 1-rank communicator): the all-reduce paths
run through RCCL and leave single-rank sketches unchanged, and every exchange
kernel of rsk_comm.hip runs: the Bloom slice-OR exchanges with its own rank
(RSK_FETCH_SELF: its slice to itself, or_rows_into_kernel, the slice back) and rsk_hll_fetch_rows with
RSK_FETCH_SELF routes owned rows through gather_rows_kernel, a self
send/recv and scatter_rows_kernel.  The N > 1 plan arithmetic is checked on
CPU (tests/test_plan.py: the library's C++ plans = shard.py's) and the
exchange plans bit-exactly with gloo at world 2 and 3 (tests/test_shard_gloo.py)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_one_rank_communicator(engine, orc):
    from redisson_amd import KeyBatch, _lib

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    from redisson_amd import shard

    _lib.check(L.rsk_comm_destroy(engine.ctx))
    assert shard.comm_info(engine) == (1, 0)  # no communicator
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    assert shard.comm_info(engine) == (1, 0)  # RCCL's own count and rank of the 1-rank communicator
    try:
        h = ctypes.c_void_p()
        _lib.check(L.rsk_hll_create(engine.ctx, 3, ctypes.byref(h)))
        keys = orc.gen_keys16(0x5EED0002, 0, 50000)
        ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
        _lib.check(L.rsk_hll_add(h, 1, ctypes.byref(ks), None))
        ref = np.zeros(16384, np.uint8)
        orc.hll_add(ref, keys, None, 16, 50000)
        _lib.check(L.rsk_hll_allreduce(h, 1))
        _lib.check(L.rsk_hll_allreduce_pool(h))
        first, count = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(L.rsk_hll_reducescatter_pool(h, ctypes.byref(first), ctypes.byref(count)))
        assert (first.value, count.value) == (0, 3)  # one rank owns the whole pool
        fetch = np.array([2, 1, 1, 0], np.uint64)  # all owned: only the count exchange runs
        _lib.check(L.rsk_hll_fetch_rows(h, fetch.ctypes.data, fetch.size))
        _lib.check(L.rsk_hll_fetch_rows(h, None, 0))
        with pytest.raises(_lib.IllegalArgumentException):  # id beyond the pool
            bad = np.array([3], np.uint64)
            _lib.check(L.rsk_hll_fetch_rows(h, bad.ctypes.data, 1))
        out = np.zeros(16384, np.uint8)
        _lib.check(L.rsk_hll_get_registers(h, 1, out.ctypes.data, _lib.RSK_MEM_HOST))
        assert np.array_equal(out, ref)
        cnt = np.zeros(1, np.uint64)
        ids = np.array([1], np.uint64)
        _lib.check(L.rsk_hll_count(h, ids.ctypes.data, 1, cnt.ctypes.data))
        assert int(cnt[0]) == orc.hll_count_dense(ref)
        b = ctypes.c_void_p()
        _lib.check(L.rsk_bloom_create(engine.ctx, 100003, 5, ctypes.byref(b)))
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
        _lib.check(L.rsk_bloom_allreduce_or(b))
        bits = np.zeros((100003 + 7) // 8, np.uint8)
        n = ctypes.c_size_t()
        _lib.check(L.rsk_bloom_export_bits(b, bits.ctypes.data, bits.size, ctypes.byref(n)))
        rb = np.zeros_like(bits)
        orc.bloom_add_batch(rb, 100003, 5, keys, None, 16, 50000, want=False)
        assert np.array_equal(bits, rb)
    finally:
        _lib.check(L.rsk_comm_destroy(engine.ctx))


def _prof(engine, name):
    return engine.prof_read(name)[1]


def test_self_exchange_runs_every_kernel(engine, orc):
    """Rows through gather -> send/recv to self -> scatter must come back
    bit-identical (an index mix-up in either kernel moves a row of another
    sketch), caches invalidated and keys created; the Bloom slice-OR of one
    rank leaves the bit string unchanged."""
    from redisson_amd import KeyBatch, _lib, shard

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    engine.prof_enable(True)
    engine.prof_reset()
    try:
        G = 6
        h = ctypes.c_void_p()
        _lib.check(L.rsk_hll_create(engine.ctx, G, ctypes.byref(h)))
        refs = []
        for g in range(G):  # distinct contents per sketch (sketch 5 stays empty)
            n = 3000 * (g + 1) if g < 5 else 0
            keys = orc.gen_keys16(0x5EED0100 + g, 0, max(n, 1))[: 16 * n]
            ref = np.zeros(16384, np.uint8)
            if n:
                ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
                _lib.check(L.rsk_hll_add(h, g, ctypes.byref(ks), None))
                orc.hll_add(ref, keys, None, 16, n)
            refs.append(ref)
        cnt = np.zeros(G, np.uint64)
        _lib.check(L.rsk_hll_count(h, None, G, cnt.ctypes.data))  # fills the caches of sketches 0..4
        shard.hll_fetch_rows(h, [4, 1, 4, 0, 5], flags=_lib.RSK_FETCH_SELF)
        assert _prof(engine, "hll_fetch_rows") == 1  # the row exchange ran (not the early exit)
        for g in range(G):
            out = np.zeros(16384, np.uint8)
            _lib.check(L.rsk_hll_get_registers(h, g, out.ctypes.data, _lib.RSK_MEM_HOST))
            assert np.array_equal(out, refs[g]), g
        ex = ctypes.c_int()
        _lib.check(L.rsk_hll_exists(h, 5, ctypes.byref(ex)))
        assert ex.value == 1  # fetched rows exist (snapshot of the owner's key)
        cnt2 = np.zeros(G, np.uint64)
        _lib.check(L.rsk_hll_count(h, None, G, cnt2.ctypes.data))
        assert [int(x) for x in cnt2] == [orc.hll_count_dense(r) for r in refs]
        # Lockstep argument errors: the bad id is reported, the communicator stays usable.
        with pytest.raises(_lib.IllegalArgumentException):
            shard.hll_fetch_rows(h, [1, G], flags=_lib.RSK_FETCH_SELF)
        shard.hll_fetch_rows(h, [2], flags=_lib.RSK_FETCH_SELF)
        with pytest.raises(_lib.IllegalArgumentException):
            _lib.check(L.rsk_hll_allreduce(h, G))
        _lib.check(L.rsk_hll_allreduce(h, 2))
        out = np.zeros(16384, np.uint8)
        _lib.check(L.rsk_hll_get_registers(h, 2, out.ctypes.data, _lib.RSK_MEM_HOST))
        assert np.array_equal(out, refs[2])
        # Bloom: the full slice-OR plan at N = 1 with the rank as its own peer
        # (odd size: the last slice is ragged).
        size, k = 1_000_003, 7
        keys = orc.gen_keys16(0x5EED0003, 0, 40000)
        b = ctypes.c_void_p()
        _lib.check(L.rsk_bloom_create(engine.ctx, size, k, ctypes.byref(b)))
        ks = KeyBatch.from_numpy(keys.reshape(-1, 16)).as_struct()
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
        _lib.check(L.rsk_bloom_allreduce_or(b))  # N = 1: nothing moves
        assert _prof(engine, "bloom_alltoall") == 0
        shard.bloom_allreduce_or(b, flags=_lib.RSK_FETCH_SELF)
        assert _prof(engine, "bloom_alltoall") == 1 and _prof(engine, "bloom_or_rows") == 1
        assert _prof(engine, "bloom_allgather") == 1
        bits = np.zeros((size + 7) // 8, np.uint8)
        n = ctypes.c_size_t()
        _lib.check(L.rsk_bloom_export_bits(b, bits.ctypes.data, bits.size, ctypes.byref(n)))
        rb = np.zeros_like(bits)
        orc.bloom_add_batch(rb, size, k, keys, None, 16, 40000, want=False)
        assert np.array_equal(bits, rb)
        _lib.check(L.rsk_bloom_destroy(b))
        _lib.check(L.rsk_hll_destroy(h))
    finally:
        engine.prof_enable(False)
        _lib.check(L.rsk_comm_destroy(engine.ctx))


def test_allreduce_without_comm_is_an_error(engine):
    from redisson_amd import IllegalArgumentException, _lib

    L = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(L.rsk_hll_create(engine.ctx, 1, ctypes.byref(h)))
    with pytest.raises(IllegalArgumentException):
        _lib.check(L.rsk_hll_allreduce(h, 0))


def test_device_memory_roundtrip(engine):
    from redisson_amd import devmem

    a = np.arange(100000, dtype=np.uint64)
    b = devmem.DeviceBuffer.from_numpy(engine, a)
    assert np.array_equal(b.to_numpy(np.uint64), a)
    b.zero()
    assert not b.to_numpy().any()
    b.free()


def _rows_equal(L, engine, a, b, G):
    """Every row of two pools equal (device copies compared in chunks)."""
    from redisson_amd import _lib

    pa, pb = L.rsk_hll_device_registers(a), L.rsk_hll_device_registers(b)
    chunk = 16384
    for lo in range(0, G, chunk):
        m = min(chunk, G - lo)
        x = np.zeros(m * 16384, np.uint8)
        y = np.zeros(m * 16384, np.uint8)
        _lib.check(L.rsk_memcpy(engine.ctx, x.ctypes.data, ctypes.c_void_p(pa + lo * 16384), x.size, 1))
        _lib.check(L.rsk_memcpy(engine.ctx, y.ctypes.data, ctypes.c_void_p(pb + lo * 16384), y.size, 1))
        if not np.array_equal(x, y):
            bad = np.nonzero((x != y).reshape(m, 16384).any(1))[0]
            return lo + int(bad[0])
    return None


@pytest.mark.parametrize("G,n", [(5000, 10_000), (100_000, 5_000_000)])
def test_routed_add_self_exchange(engine, orc, G, n):
    """rsk_hll_add_grouped_routed on a 1-rank communicator with RSK_FETCH_SELF:
    the route count and scatter kernels, the record exchange through RCCL to
    itself and the record-input grouped add (the direct CAS kernel for the
    small batch, the partitioned pipeline for the large one, onto a pending
    clear) give the registers of the plain grouped add; ids >= G are ignored."""
    from redisson_amd import _lib, devmem, shard
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    engine.prof_enable(True)
    engine.prof_reset()
    try:
        groups, keys = orc.gen_grouped(0x5EED0006, G, 0, n)
        groups[::101] = G + 7
        kd = devmem.DeviceBuffer.from_numpy(engine, keys)
        gd = devmem.DeviceBuffer.from_numpy(engine, groups)
        kb = kd.keys_fixed(n, 16)
        a = GroupedHyperLogLog(engine, G)
        b = GroupedHyperLogLog(engine, G)
        a.add(kb, gd)
        a.add(kb, gd)  # (rows to clear below)
        b.clear()
        b.add(kb, gd)  # reference: the plain grouped add from a cleared pool
        a.clear()      # the routed add completes the lazy clear on the owned rows
        assert shard.hll_add_grouped_routed(a.pool, kb, gd, flags=_lib.RSK_FETCH_SELF) == (0, G)
        assert _prof(engine, "hll_route_exchange") == 1
        assert _rows_equal(L, engine, a.pool, b.pool, G) is None
        for gid in (0, 1, G // 2, G - 1):
            ref = np.zeros(16384, np.uint8)
            sel = groups == gid
            orc.hll_add(ref, keys.reshape(-1, 16)[sel].reshape(-1), None, 16, int(sel.sum()))
            assert np.array_equal(a.registers(gid), ref), gid
        assert list(a.count(ids=[0, 1])) == list(b.count(ids=[0, 1]))
        shard.hll_add_grouped_routed(a.pool, kb, gd)  # without the flag: own records stay local; re-adds change nothing
        assert _rows_equal(L, engine, a.pool, b.pool, G) is None
        a.close()
        b.close()
        kd.free()
        gd.free()
    finally:
        engine.prof_enable(False)
        _lib.check(L.rsk_comm_destroy(engine.ctx))


def _assert_pool_equals_oracle(L, engine, orc, pool, G, n, zipf, seed=0x5EED0006):
    """Every row of a full-size pool against the oracle over the whole pair
    stream (16 GB at 1M sketches, compared in 1 GiB chunks)."""
    import os

    from redisson_amd import _lib

    thr = max(1, min(16, os.cpu_count() or 1))
    groups = orc.gen_grouped_zipf_groups(seed, G, zipf, 0, n, thr) if zipf else orc.gen_grouped_groups(seed, G, 0, n, thr)
    ref = np.zeros((G, 16384), np.uint8)
    orc.hll_add_keys_by_groups(ref, G, groups, seed, 0, thr)
    del groups
    base = L.rsk_hll_device_registers(pool)
    chunk = 65536
    buf = np.empty((chunk, 16384), np.uint8)
    bad = []
    for lo in range(0, G, chunk):
        m = min(chunk, G - lo)
        _lib.check(L.rsk_memcpy(engine.ctx, buf.ctypes.data, ctypes.c_void_p(base + lo * 16384), m * 16384, 1))
        bad.extend((np.nonzero((buf[:m] != ref[lo:lo + m]).any(1))[0] + lo)[:16].tolist())
    assert not bad, (len(bad), bad[:16])
    return ref


def test_routed_add_c5_full_size_self_exchange(engine, orc):
    """BASELINE configs[4] at its per-GPU size through the routed form at N = 1
    (every record through RCCL to itself): every sketch is bit-exact against
    the oracle over the whole pair stream."""
    from redisson_amd import _lib, devmem, shard
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    try:
        G, n = 1_000_000, 500_000_000
        g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
        pool = GroupedHyperLogLog(engine, G)
        pool.clear()
        assert shard.hll_add_grouped_routed(pool.pool, k.keys_fixed(n, 16), g, flags=_lib.RSK_FETCH_SELF) == (0, G)
        g.free()
        k.free()
        _assert_pool_equals_oracle(L, engine, orc, pool.pool, G, n, 0.0)  # every sketch
        pool.close()
        _lib.check(L.rsk_trim(engine.ctx))
    finally:
        _lib.check(L.rsk_comm_destroy(engine.ctx))


def _all_rows(L, engine, pool, G):
    """The whole pool as a [G][16384] host array (rsk_hll_device_registers first
    completes any pending clear)."""
    from redisson_amd import _lib

    p = L.rsk_hll_device_registers(pool)
    assert p
    out = np.zeros((G, 16384), np.uint8)
    _lib.check(L.rsk_memcpy(engine.ctx, out.ctypes.data, ctypes.c_void_p(p), out.size, 1))
    return out


@pytest.mark.parametrize("G,n,vrank", [(5000, 10_000, 1), (100_003, 5_000_000, 1), (100_003, 5_000_000, 2)])
def test_routed_add_owned_subrange(engine, orc, route, G, n, vrank):
    """the routed add on an owned SUB-range (rank vrank of 3, planned
    on the 1-rank communicator by the route_vranks test route: records of the
    other owners dropped): the owned rows equal the plain grouped add's (the
    d_regs + first * 16384 and PCount offsets), and after a clear every row
    outside the owned range reads as cleared -- per row (registers, PFCOUNT,
    exists), through countWith / mergeWith members, through a fetch, and for the
    whole pool -- never the registers it held before the clear."""
    from redisson_amd import _lib, devmem, shard
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    try:
        groups, keys = orc.gen_grouped(0x5EED0006, G, 0, n)
        kd = devmem.DeviceBuffer.from_numpy(engine, keys)
        gd = devmem.DeviceBuffer.from_numpy(engine, groups)
        kb = kd.keys_fixed(n, 16)
        first, count = shard.owned_range(G, 3, vrank)
        assert count > 0 and first > 0
        a = GroupedHyperLogLog(engine, G)
        b = GroupedHyperLogLog(engine, G)
        b.clear()
        b.add(kb, gd)  # reference: every row from the plain grouped add
        ref = _all_rows(L, engine, b.pool, G)
        a.add(kb, gd)  # a's rows all hold registers before the clear
        a.clear()
        route(route_vranks=3, route_vrank=vrank)
        assert shard.hll_add_grouped_routed(a.pool, kb, gd, flags=_lib.RSK_FETCH_SELF) == (first, count)
        out_lo, out_hi = first - 1, (first + count) % G  # rows just outside the owned range
        for gid in (first, first + count - 1, first + count // 2):
            assert np.array_equal(a.registers(gid), ref[gid]), gid
        for gid in (0, out_lo, out_hi):
            assert not a.registers(gid).any(), gid  # cleared, not the pre-clear registers
            ex = ctypes.c_int()
            _lib.check(L.rsk_hll_exists(a.pool, gid, ctypes.byref(ex)))
            assert ex.value == 0
        assert list(a.count(ids=[out_lo, first])) == [0, int(b.count(ids=[first])[0])]
        # countWith of an owned row with a pending one = the owned row alone
        cw = a.countWith(np.array([[first, out_hi]], np.uint64))
        assert int(cw[0]) == int(b.count(ids=[first])[0])
        # a second routed add onto the owned rows (pending rows elsewhere): re-adds change nothing
        shard.hll_add_grouped_routed(a.pool, kb, gd)
        assert np.array_equal(a.registers(first), ref[first])
        # mergeWith into a pending row: the source's registers, not a max with stale ones
        a.mergeWith(np.array([out_lo], np.uint64), np.array([first], np.uint64))
        assert np.array_equal(a.registers(out_lo), ref[first])
        route(route_vranks=0)
        # a fetch (N = 1: every row owned) leaves the pending rows cleared too
        shard.hll_fetch_rows(a.pool, [out_hi, first], flags=_lib.RSK_FETCH_SELF)
        assert not a.registers(out_hi).any()
        whole = _all_rows(L, engine, a.pool, G)
        owned = np.zeros(G, bool)
        owned[first:first + count] = True
        assert np.array_equal(whole[owned], ref[owned])
        rest = ~owned
        rest[out_lo] = False  # the mergeWith destination
        assert not whole[rest].any()
        a.close()
        b.close()
        kd.free()
        gd.free()
    finally:
        route(route_vranks=0)
        _lib.check(L.rsk_comm_destroy(engine.ctx))


@pytest.mark.parametrize("G,n,heavy,vranks,vrank,self_", [
    (100_003, 5_000_000, 64, 0, 0, True),     # every heavy row through RCCL to itself
    (100_003, 5_000_000, 64, 3, 1, False),    # owner 1 of 3: heavy groups of ranks 0 / 2 are rows (dropped with
                                              # their records), its own groups stay records
    (100_003, 5_000_000, 300, 3, 0, True),    # owner 0 of 3, rows through RCCL (the Zipf-hot range)
    (20_000, 8_000_000, 0, 0, 0, True),       # auto: >= 2048 pairs per heavy group at >= 2^22 pairs
])
def test_routed_add_heavy_precombine(engine, orc, route, G, n, heavy, vranks, vrank, self_):
    """VERDICT r05 Next 2: under Zipf(1.1) the groups with many pairs are folded
    into 16 KiB rows where the pairs are, the rows (not the records) go to the
    owner, which max-merges them after its own apply.  The owned rows must equal
    the plain grouped add's, bit for bit, whichever groups the sample makes heavy;
    the pre-combine ran (its stages were timed)."""
    from redisson_amd import _lib, devmem, shard
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    engine.prof_enable(True)
    engine.prof_reset()
    try:
        if heavy:
            groups, keys = orc.gen_grouped_zipf(0x5EED0006, G, 1.1, 0, n)
        else:
            groups, keys = orc.gen_grouped(0x5EED0006, G, 0, n)  # 400 pairs per group: none heavy ...
            groups[: n // 4] = np.arange(n // 4, dtype=np.uint32) % 64  # ... but 64 groups of ~31k pairs
        kd = devmem.DeviceBuffer.from_numpy(engine, keys)
        gd = devmem.DeviceBuffer.from_numpy(engine, groups)
        kb = kd.keys_fixed(n, 16)
        first, count = shard.owned_range(G, vranks or 1, vrank)
        b = GroupedHyperLogLog(engine, G)
        b.clear()
        b.add(kb, gd)
        ref = _all_rows(L, engine, b.pool, G)
        a = GroupedHyperLogLog(engine, G)
        a.add(kb, gd)  # stale rows under the clear
        a.clear()
        route(route_heavy=heavy, route_vranks=vranks, route_vrank=vrank)
        flags = _lib.RSK_FETCH_SELF if self_ else 0
        assert shard.hll_add_grouped_routed(a.pool, kb, gd, flags=flags) == (first, count)
        assert _prof(engine, "hll_route_heavy") == 1
        assert _prof(engine, "hll_route_heavy_rows") == 1  # some group was heavy
        assert _prof(engine, "hll_route_rows_merge") == 1
        got = _all_rows(L, engine, a.pool, G)
        bad = np.nonzero((got[first:first + count] != ref[first:first + count]).any(1))[0]
        assert bad.size == 0, (bad.size, (bad[:10] + first).tolist())
        assert not got[:first].any() and not got[first + count:].any()  # outside: cleared
        # PFCOUNT of owned rows: merged rows' precomputed estimates were retired
        ids = np.array([first, first + 1, first + 2, first + count - 1], np.uint64)
        assert list(a.count(ids=ids)) == list(b.count(ids=ids))
        a.close()
        b.close()
        kd.free()
        gd.free()
    finally:
        route(route_vranks=0, route_heavy=0)
        engine.prof_enable(False)
        _lib.check(L.rsk_comm_destroy(engine.ctx))


def test_routed_add_c5_zipf_full_size_heavy_rows(engine, orc):
    """BASELINE configs[4]'s Zipf(1.1) stress variant at its per-GPU size (1M
    sketches, 500M pairs) through the routed add on one GPU with the self
    exchange: the automatic heavy-group pre-combine folds the ~12k sketches of
    >= 2048 pairs into rows (which then travel through RCCL to the owner and are
    max-merged), the rest go as records.  Every sketch is bit-exact against
    the oracle over the whole stream, and the PFCOUNTs of the 64 hottest (heavy
    rows: the merged rows' precomputed estimates retired)."""

    from redisson_amd import _lib, devmem, shard
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    engine.prof_enable(True)
    engine.prof_reset()
    try:
        G, n = 1_000_000, 500_000_000
        g, k = devmem.gen_grouped_zipf(engine, 0x5EED0006, G, 1.1, 0, n)
        pool = GroupedHyperLogLog(engine, G)
        pool.clear()
        assert shard.hll_add_grouped_routed(pool.pool, k.keys_fixed(n, 16), g, flags=_lib.RSK_FETCH_SELF) == (0, G)
        assert _prof(engine, "hll_route_heavy_rows") == 1
        g.free()
        k.free()
        ref = _assert_pool_equals_oracle(L, engine, orc, pool.pool, G, n, 1.1)  # every sketch
        cnt = pool.count(ids=list(range(64)))
        assert [int(c) for c in cnt] == [orc.hll_count_dense(ref[i]) for i in range(64)]
        pool.close()
        _lib.check(L.rsk_trim(engine.ctx))
    finally:
        engine.prof_enable(False)
        _lib.check(L.rsk_comm_destroy(engine.ctx))


@pytest.mark.parametrize("G,n,heavy,vranks,vrank", [
    (200_003, 6_000_000, 2, 0, 0),   # nearly every group heavy: the 65536-row cap cuts the heavy set (by id)
    (10, 300_000, 64, 3, 2),         # the tail owner (10 = 3 + 3 + 4), every group heavy
    (2, 50_000, 64, 3, 0),           # G < N: ranks 0, 1 own nothing; rank 2 owns both
])
def test_routed_add_heavy_edges(engine, orc, route, G, n, heavy, vranks, vrank):
    """The heavy pre-combine at its edges: the per-call cap on heavy rows (the
    groups past it stay records), the tail owner, and a rank that owns no
    sketch (its pairs all go elsewhere as rows or records).  Owned rows equal
    the plain grouped add's."""
    from redisson_amd import _lib, devmem, shard
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid))
    try:
        groups, keys = orc.gen_grouped(0x5EED0016, G, 0, n)
        kd = devmem.DeviceBuffer.from_numpy(engine, keys)
        gd = devmem.DeviceBuffer.from_numpy(engine, groups)
        kb = kd.keys_fixed(n, 16)
        b = GroupedHyperLogLog(engine, G)
        b.clear()
        b.add(kb, gd)
        ref = _all_rows(L, engine, b.pool, G)
        a = GroupedHyperLogLog(engine, G)
        a.clear()
        route(route_heavy=heavy, route_vranks=vranks, route_vrank=vrank)
        first, count = shard.owned_range(G, vranks or 1, vrank)
        assert shard.hll_add_grouped_routed(a.pool, kb, gd, flags=_lib.RSK_FETCH_SELF) == (first, count)
        route(route_vranks=0, route_heavy=0)
        got = _all_rows(L, engine, a.pool, G)
        assert np.array_equal(got[first:first + count], ref[first:first + count])
        assert not got[:first].any() and not got[first + count:].any()
        a.close()
        b.close()
        kd.free()
        gd.free()
    finally:
        route(route_vranks=0, route_heavy=0)
        _lib.check(L.rsk_comm_destroy(engine.ctx))
