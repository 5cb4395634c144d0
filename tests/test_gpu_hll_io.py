"""Batched Redis strings of an HLL pool (rsk_hll_export_redis_batch /
rsk_hll_import_redis_batch, rsk_hll_io.hip): the checkpoint path of SURVEY 5.
The batch GET must equal the per-key GET (rsk_hll_export_redis) byte for byte
in every encoding state, and the oracle's encoders on the registers; the batch
SET must equal the per-key SET, reject what it rejects with nothing changed,
and round-trip a whole pool."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_C2 = 0x5EED0002


@pytest.fixture(scope="module")
def L():
    from redisson_amd import _lib

    return _lib.load()


def _pool(L, engine, n):
    from redisson_amd import _lib

    h = ctypes.c_void_p()
    _lib.check(L.rsk_hll_create(engine.ctx, n, ctypes.byref(h)))
    return h


def _regs(L, h, i):
    from redisson_amd import _lib

    out = np.zeros(16384, np.uint8)
    _lib.check(L.rsk_hll_get_registers(h, i, out.ctypes.data, _lib.RSK_MEM_HOST))
    return out


def _export1(L, h, i):
    from redisson_amd import _lib

    buf = (ctypes.c_uint8 * 12304)()
    n = ctypes.c_size_t()
    _lib.check(L.rsk_hll_export_redis(h, i, buf, 12304, ctypes.byref(n)))
    return bytes(buf[: n.value])


def _export_batch(L, h, ids, cap=None):
    from redisson_amd import _lib

    ids = np.ascontiguousarray(ids, np.uint64)
    offs = np.zeros(ids.size + 1, np.uint64)
    cap = ids.size * 12304 if cap is None else cap
    out = np.zeros(max(1, cap), np.uint8)
    rc = L.rsk_hll_export_redis_batch(h, ids.ctypes.data, ids.size, out.ctypes.data, cap, offs.ctypes.data)
    return rc, out, offs


def _strings(out, offs):
    return [bytes(out[int(offs[i]):int(offs[i + 1])]) for i in range(offs.size - 1)]


def _import_batch(L, h, ids, strs):
    ids = np.ascontiguousarray(ids, np.uint64)
    offs = np.zeros(len(strs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(s) for s in strs])
    data = np.frombuffer(b"".join(strs) or b"\0", np.uint8).copy()
    return L.rsk_hll_import_redis_batch(h, ids.ctypes.data, ids.size, data.ctypes.data, offs.ctypes.data)


def _mixed_pool(L, engine, orc):
    """A pool holding every encoding state: missing, fresh (PFADD of nothing),
    sparse at several sizes, promoted by size (> 3000 bytes) and by a register
    above 32, PFMERGE destinations, SET of canonical / non-canonical sparse and
    of dense strings (one with non-zero unused header bytes)."""
    from redisson_amd import KeyBatch, _lib

    G = 64
    h = _pool(L, engine, G)
    keys = orc.gen_keys16(SEED_C2, 0, 60000).reshape(-1, 16)

    def add(i, ks):
        ch = ctypes.c_uint8()
        ks_ = KeyBatch.from_numpy(ks).as_struct()
        _lib.check(L.rsk_hll_add(h, i, ctypes.byref(ks_), ctypes.byref(ch)))

    # ids 30 .. 63: grouped adds of a few keys each (the C5 shape; first: a grouped add
    # drops every kept SET string of the pool)
    gk = orc.gen_keys16(SEED_C2, 100000, 34 * 300).reshape(-1, 16)
    grp = (30 + np.arange(gk.shape[0]) % 34).astype(np.uint32)
    ks_ = KeyBatch.from_numpy(gk).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks_), grp.ctypes.data))
    add(1, keys[:0])                     # created, all-zero: one XZERO
    sizes = [1, 2, 5, 17, 64, 100, 300, 700, 1200, 2000, 5000, 20000]
    at = 0
    for j, m in enumerate(sizes):        # ids 2 .. 13: sparse, then promoted by size
        add(2 + j, keys[at:at + m])
        at += m
    # id 20: a register above 32 (a crafted dense string), then SET sparse strings
    raw = np.zeros(16384, np.uint8)
    raw[100] = 40
    raw[101:140] = 3
    dense = orc.hll_encode_dense(raw)
    b = (ctypes.c_uint8 * len(dense)).from_buffer_copy(dense)
    _lib.check(L.rsk_hll_import_redis(h, 20, b, len(dense)))
    # id 21: PFMERGE destination (dense even when small)
    pools = (ctypes.c_void_p * 1)(h.value)
    src = (ctypes.c_uint64 * 1)(3)
    _lib.check(L.rsk_hll_merge(h, 21, pools, src, 1))
    # id 22: canonical sparse SET; id 23: non-canonical (a VAL run cut 2 + 2, two ZEROs in a row)
    r2 = np.zeros(16384, np.uint8)
    r2[10:14] = 5
    canon = orc.hll_encode_sparse(r2)
    b = (ctypes.c_uint8 * len(canon)).from_buffer_copy(canon)
    _lib.check(L.rsk_hll_import_redis(h, 22, b, len(canon)))
    hdr = bytes(canon[:16])
    # registers 0-9 zero (ZERO 5 + ZERO 5), 10-13 = 5 (VAL 2 + VAL 2), 14.. zero (XZERO)
    body = bytes([4, 4, 0x80 | (4 << 2) | 1, 0x80 | (4 << 2) | 1])
    rest = 16384 - 14
    body += bytes([0x40 | ((rest - 1) >> 8), (rest - 1) & 0xFF])
    nonc = hdr + body
    b = (ctypes.c_uint8 * len(nonc)).from_buffer_copy(nonc)
    _lib.check(L.rsk_hll_import_redis(h, 23, b, len(nonc)))
    # id 24: dense SET with a non-zero unused header byte (kept as SET)
    d2 = bytearray(orc.hll_encode_dense(r2))
    d2[6] = 7
    b = (ctypes.c_uint8 * len(d2)).from_buffer_copy(bytes(d2))
    _lib.check(L.rsk_hll_import_redis(h, 24, b, len(d2)))
    return h, G


def test_export_batch_equals_per_key(L, engine, orc):
    """Every encoding state: the batch GET of all ids (in a shuffled order, with
    repeats) equals the per-key GET of each, including the encoding decision
    (promotion) and the card bytes after a PFCOUNT; missing keys are empty."""
    from redisson_amd import _lib

    h, G = _mixed_pool(L, engine, orc)
    cnt = np.zeros(4, np.uint64)
    ids4 = np.array([2, 7, 22, 23], np.uint64)
    _lib.check(L.rsk_hll_count(h, ids4.ctypes.data, 4, cnt.ctypes.data))  # card caches refreshed
    rng = np.random.default_rng(3)
    ids = np.concatenate([rng.permutation(G), rng.integers(0, G, 40)]).astype(np.uint64)
    rc, out, offs = _export_batch(L, h, ids)
    assert rc == 0
    got = _strings(out, offs)
    want = [_export1(L, h, int(i)) for i in ids]
    assert got == want
    assert got[list(ids).index(0)] == b""  # never written
    enc = {int(i): s[4] for i, s in zip(ids, got) if s}
    assert enc[1] == 1 and enc[2] == 1 and enc[13] == 0 and enc[20] == 0 and enc[21] == 0 and enc[23] == 1
    # the non-canonical SET string comes back as it was SET (card bytes as PFCOUNT left them)
    s23 = got[list(ids).index(23)]
    assert s23[16:] == bytes([4, 4, 0x91, 0x91, 0x7F, 0xF1])
    L.rsk_hll_destroy(h)


def test_export_batch_matches_oracle_encoders(L, engine, orc):
    """The device encoders against the oracle's (orc_hll_encode_sparse / _dense)
    on the same registers, for sparse and dense keys."""
    h, G = _mixed_pool(L, engine, orc)
    ids = np.array([1, 2, 3, 5, 8, 11, 12, 13, 21, 30, 45, 63], np.uint64)
    rc, out, offs = _export_batch(L, h, ids)
    assert rc == 0
    for i, s in zip(ids.tolist(), _strings(out, offs)):
        regs = _regs(L, h, i)
        card = s[8:16]
        ref = orc.hll_encode_sparse(regs, card) if s[4] == 1 else orc.hll_encode_dense(regs, card)
        assert s == ref, i
    L.rsk_hll_destroy(h)


def _row_with_sparse_len(orc, target):
    """Registers whose canonical sparse string is exactly target bytes: N
    single-register VALs with a ZERO of 4 between each two, one of them a run
    of 5 (VAL 4 + VAL 1) for an even target, and an XZERO tail."""
    extra = (target - 17) % 2  # header 16 + N VALs + (N - 1) ZEROs + the XZERO tail's 2
    n = (target - 17 - extra) // 2
    r = np.zeros(16384, np.uint8)
    j = 0
    for k in range(n):
        run = 5 if (extra and k == 0) else 1
        r[j:j + run] = 1 + k % 32
        j += run + 4
    assert len(orc.hll_encode_sparse(r)) == target
    return r


def test_export_sparse_length_boundary(L, engine, orc):
    """The encoder's sparse-or-dense decision at the 3000-byte limit
    (server.hll_sparse_max_bytes): rows of 2996 .. 3000 sparse bytes come back
    sparse; single PFADDs then grow them across the limit -- each GET equals
    the per-key GET and the oracle's encoder for the encoding it chose, sparse
    exactly while the canonical sparse string fits (promotion is for good)."""
    from redisson_amd import KeyBatch, _lib

    targets = [2996, 2997, 2999, 3000]
    rows = [_row_with_sparse_len(orc, t) for t in targets]
    strs = [orc.hll_encode_sparse(r) for r in rows]
    h = _pool(L, engine, len(rows))
    ids = np.arange(len(rows), dtype=np.uint64)
    assert _import_batch(L, h, ids, strs) == 0
    rc, out, offs = _export_batch(L, h, ids)
    assert rc == 0 and _strings(out, offs) == strs
    keys = orc.gen_keys16(SEED_C2, 500000, 16 * len(rows)).reshape(len(rows), 16, 16)
    promoted = [False] * len(rows)
    for step in range(16):
        for i in range(len(rows)):
            ch = ctypes.c_uint8()
            ks_ = KeyBatch.from_numpy(np.ascontiguousarray(keys[i, step:step + 1])).as_struct()
            _lib.check(L.rsk_hll_add(h, i, ctypes.byref(ks_), ctypes.byref(ch)))
        rc, out, offs = _export_batch(L, h, ids)
        assert rc == 0
        for i, s in enumerate(_strings(out, offs)):
            regs = _regs(L, h, i)
            sp = orc.hll_encode_sparse(regs, s[8:16])
            promoted[i] = promoted[i] or len(sp) > 3000
            assert s[4] == (0 if promoted[i] else 1), (step, i, len(sp))
            assert s == (orc.hll_encode_dense(regs, s[8:16]) if promoted[i] else sp), (step, i)
            assert s == _export1(L, h, i), (step, i)
    assert all(promoted)
    L.rsk_hll_destroy(h)


def test_export_batch_small_buffer(L, engine, orc):
    """cap below the total: RSK_ERR_INVALID_ARG, offsets[n] = the bytes needed,
    nothing written; then the exact size succeeds."""
    from redisson_amd import _lib

    h, G = _mixed_pool(L, engine, orc)
    ids = np.arange(G, dtype=np.uint64)
    rc, out, offs = _export_batch(L, h, ids, cap=100)
    assert rc == _lib.RSK_ERR_INVALID_ARG and int(offs[-1]) > 100
    assert not out[:100].any()
    need = int(offs[-1])
    rc, out2, offs2 = _export_batch(L, h, ids, cap=need)
    assert rc == 0 and int(offs2[-1]) == need
    L.rsk_hll_destroy(h)


def test_export_batch_chunks_and_late_overflow(L, engine, orc):
    """More keys than one encode chunk (16384 keys, then 65536 per chunk): the
    chunked export equals the per-key GET at the chunk edges, and a cap one
    byte short of the total fails with offsets[n] = the bytes needed, the
    first chunk's strings written."""
    from redisson_amd import KeyBatch, _lib

    G = 70000
    h = _pool(L, engine, G)
    gk = orc.gen_keys16(SEED_C2, 0, 4 * G).reshape(-1, 16)
    grp = (np.arange(gk.shape[0]) % G).astype(np.uint32)
    grp[:40000] = 0  # one key with many pairs (dense by size); every key keeps a pair
    assert np.unique(grp).size == G
    ks_ = KeyBatch.from_numpy(gk).as_struct()
    _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks_), grp.ctypes.data))
    ids = np.arange(G, dtype=np.uint64)
    rc, out, offs = _export_batch(L, h, ids, cap=G * 300)
    assert rc == 0
    need = int(offs[-1])
    got = _strings(out, offs)
    for i in (0, 1, 16383, 16384, 65535, 65536, 65537, G - 1):
        assert got[i] == _export1(L, h, i), i
    rc2, out2, offs2 = _export_batch(L, h, ids, cap=need - 1)
    assert rc2 == _lib.RSK_ERR_INVALID_ARG and int(offs2[-1]) == need
    assert np.array_equal(offs2, offs)
    first = int(offs[16384])
    assert np.array_equal(out2[:first], out[:first])
    L.rsk_hll_destroy(h)


def test_import_batch_round_trip(L, engine, orc):
    """Export every key of the mixed pool, import the strings into a fresh pool
    in one call: same registers, same GET bytes (kept SET strings included),
    same encodings; the import equals the per-key SET of the same strings."""
    h, G = _mixed_pool(L, engine, orc)
    ids = np.arange(G, dtype=np.uint64)
    rc, out, offs = _export_batch(L, h, ids)
    assert rc == 0
    strs = _strings(out, offs)
    present = [i for i in range(G) if strs[i]]
    h2 = _pool(L, engine, G)
    assert _import_batch(L, h2, present, [strs[i] for i in present]) == 0
    h3 = _pool(L, engine, G)
    for i in present:
        b = (ctypes.c_uint8 * len(strs[i])).from_buffer_copy(strs[i])
        assert L.rsk_hll_import_redis(h3, i, b, len(strs[i])) == 0
    for i in present:
        assert np.array_equal(_regs(L, h2, i), _regs(L, h, i)), i
    rc2, out2, offs2 = _export_batch(L, h2, ids)
    rc3, out3, offs3 = _export_batch(L, h3, ids)
    assert rc2 == 0 and rc3 == 0
    assert _strings(out2, offs2) == strs == _strings(out3, offs3)
    for x in (h, h2, h3):
        L.rsk_hll_destroy(x)


def test_import_batch_rejects_with_nothing_changed(L, engine, orc):
    """A corrupt string anywhere in the batch (bad magic, wrong dense length,
    sparse opcodes covering too few / too many registers, an XZERO cut by the
    end) fails the call with the per-key error code; no key changes.  A key SET
    twice keeps the later string."""
    from redisson_amd import _lib

    r = np.zeros(16384, np.uint8)
    r[5] = 3
    good = orc.hll_encode_sparse(r)
    hdr = good[:16]
    bad = {
        "magic": (b"HYLX" + good[4:], _lib.RSK_ERR_WRONGTYPE),
        "dense_len": (b"HYLL\x00" + good[5:16] + bytes(100), _lib.RSK_ERR_WRONGTYPE),
        "short": (hdr + bytes([0x7F]), _lib.RSK_ERR_INVALID_HLL),                  # 64 registers only
        "long": (good + bytes([0x00]), _lib.RSK_ERR_INVALID_HLL),                  # one register too many
        "cut_xzero": (hdr + bytes([0x00, 0x40]), _lib.RSK_ERR_INVALID_HLL),        # XZERO without its second byte
    }
    for name, (s, code) in bad.items():
        h = _pool(L, engine, 8)
        assert _import_batch(L, h, [1, 2, 3], [good, s, good]) == code, name
        assert _export_batch(L, h, np.arange(8))[2][-1] == 0, name  # nothing exists
        L.rsk_hll_destroy(h)
    h = _pool(L, engine, 8)
    r2 = r.copy()
    r2[9] = 7
    later = orc.hll_encode_sparse(r2)
    assert _import_batch(L, h, [4, 4, 5], [good, later, good]) == 0
    assert np.array_equal(_regs(L, h, 4), r2) and np.array_equal(_regs(L, h, 5), r)
    L.rsk_hll_destroy(h)


def test_import_batch_late_failure_restores_every_row(L, engine, orc):
    """The batched SET decodes each upload chunk as soon as it is checked, with
    the rows it replaces copied aside: a corrupt string in the LAST chunk must
    still leave every key as it was -- registers, card bytes and GET bytes of
    all 20000 keys equal to before the call -- and the same batch without the
    corrupt string then lands whole."""
    from redisson_amd import _lib

    rng = np.random.default_rng(41)
    n = 20000

    def strings(seed_shift):
        out = []
        for i in range(n):
            r = np.zeros(16384, np.uint8)
            idx = rng.integers(0, 16384, size=int(rng.integers(1, 40)))
            r[idx] = rng.integers(1, 20, size=idx.size)
            out.append(bytes(orc.hll_encode_sparse(r)))
        return out

    first = strings(0)
    h = _pool(L, engine, n)
    ids = np.arange(n)
    assert _import_batch(L, h, ids, first) == 0
    rc, out0, offs0 = _export_batch(L, h, ids)
    assert rc == 0
    before = [_regs(L, h, i).copy() for i in (0, 1, n // 2, n - 2)]
    second = strings(1)
    bad = second[-1] + bytes([0x00])  # one register too many, at the very end of the batch
    assert _import_batch(L, h, ids, second[:-1] + [bad]) == _lib.RSK_ERR_INVALID_HLL
    rc, out1, offs1 = _export_batch(L, h, ids)
    assert rc == 0 and np.array_equal(offs1, offs0) and np.array_equal(out1, out0)  # every key as it was
    for j, i in enumerate((0, 1, n // 2, n - 2)):
        assert np.array_equal(_regs(L, h, i), before[j]), i
    assert _import_batch(L, h, ids, second) == 0
    rc, out2, offs2 = _export_batch(L, h, ids)
    assert rc == 0 and _strings(out2, offs2) == second
    L.rsk_hll_destroy(h)


def test_import_batch_every_sparse_shape(L, engine, orc):
    """Registers with runs of every opcode length at 64-byte step boundaries:
    XZERO second bytes in lane 63 and lane 0, runs of 1..4 VALs, zero runs of
    1..64 and 65..16384 -- decoded exactly; GET returns the same bytes (the
    canonical strings re-encoded, those over 3000 bytes kept as SET)."""
    rng = np.random.default_rng(17)
    strs, regs = [], []
    for t in range(48):
        r = np.zeros(16384, np.uint8)
        j = int(rng.integers(0, 200))
        while j < 16384:
            run = int(rng.integers(1, 9))
            r[j:j + run] = int(rng.integers(1, 33))
            j += run + int(rng.choice([1, 2, 63, 64, 65, 66, 130, 300]))
            if rng.random() < 0.05:
                j += int(rng.integers(1000, 4000))
        s = orc.hll_encode_sparse(r)
        strs.append(s)
        regs.append(r)
    h = _pool(L, engine, len(strs))
    assert _import_batch(L, h, np.arange(len(strs)), strs) == 0
    rc, out, offs = _export_batch(L, h, np.arange(len(strs)))
    assert rc == 0
    for i in range(len(strs)):
        assert np.array_equal(_regs(L, h, i), regs[i]), i
    assert _strings(out, offs) == strs  # canonical ones re-encoded, longer ones kept as SET (as per key)
    L.rsk_hll_destroy(h)


def test_import_batch_long_sparse(L, engine, orc):
    """Sparse strings longer than the decoder's 4 KiB LDS stage (parsed from
    global memory) next to staged ones: 16384 single-register VALs (16400
    bytes), a 5000-byte one, a 4096-byte payload (the stage's edge, staged)
    and 4097 (not) -- decoded exactly and kept as SET; one covering a
    register too many fails the whole batch with nothing written."""
    from redisson_amd import _lib

    def hdr():
        return bytearray(b"HYLL\x01" + bytes(11))

    rows, strs = [], []
    r = (1 + np.arange(16384) % 2).astype(np.uint8)  # 1, 2, 1, 2, ...: one VAL per register
    rows.append(r)
    for plen in (5000, 4096, 4097, 3001):
        # plen - 1 single-register VALs alternating 3 / 4, then one XZERO... sized to plen bytes
        nv = plen - 2
        rr = np.zeros(16384, np.uint8)
        rr[:nv] = 3 + np.arange(nv) % 2
        rows.append(rr)
    for rr in rows:
        sp = orc.hll_encode_sparse(rr)
        strs.append(bytes(sp))
    assert [len(x) - 16 for x in strs] == [16384, 5000, 4096, 4097, 3001]
    h = _pool(L, engine, len(strs) + 1)
    ids = np.arange(len(strs))
    assert _import_batch(L, h, ids, strs) == 0
    for i, rr in enumerate(rows):
        assert np.array_equal(_regs(L, h, i), rr), i
    rc, out, offs = _export_batch(L, h, ids)
    assert rc == 0 and _strings(out, offs) == strs  # kept as SET (over 3000 bytes)
    # one register too many (a trailing ZERO 1) on the long, unstaged form: nothing is written
    bad = strs[0] + bytes([0x00])
    before = _regs(L, h, 5).copy()
    assert _import_batch(L, h, np.array([5, 0]), [strs[1], bad]) == _lib.RSK_ERR_INVALID_HLL
    assert np.array_equal(_regs(L, h, 5), before)
    L.rsk_hll_destroy(h)


@pytest.mark.parametrize("pin,copy", [(0, 0), (-1, 0), (0, -1), (-1, -1)])
def test_dense_pool_round_trip_many_pieces(L, engine, orc, route, pin, copy):
    """70000 dense keys (861 MB of strings): one export chunk is ~806 MB, so
    the staged copy-out (route io_pin = -1) cycles its ring of pinned slots
    several times, or the output buffer is pinned for the call and takes the
    DMA (the default for a buffer >= 256 MiB), the DMAs on the measured SDMA
    engine (route io_engine = 0) or HIP's copies (-1); the import stages
    ~861 MB in pieces; SET then GET returns the same bytes, and the registers
    equal the oracle's decode."""
    route(io_pin=pin, io_engine=copy)
    rng = np.random.default_rng(29)
    G = 70000
    rows = rng.integers(0, 25, size=(64, 16384), dtype=np.uint8)
    strs64 = [bytes(orc.hll_encode_dense(r)) for r in rows]
    assert all(len(x) == 12304 for x in strs64)
    pick = rng.integers(0, 64, G)
    strs = [strs64[j] for j in pick]
    h = _pool(L, engine, G)
    ids = np.arange(G)
    assert _import_batch(L, h, ids, strs) == 0
    rc, out, offs = _export_batch(L, h, ids)
    assert rc == 0
    assert int(offs[-1]) == 12304 * G
    assert np.array_equal(out[: 12304 * G].reshape(G, 12304), np.frombuffer(b"".join(strs), np.uint8).reshape(G, 12304))
    for i in (0, 1, 65535, 65536, G - 1):
        assert np.array_equal(_regs(L, h, i), rows[pick[i]]), i
    L.rsk_hll_destroy(h)


def test_c5_pool_checkpoint_round_trip(L, engine, orc):
    """BASELINE configs[4] per GPU: 1M sketches after 500M grouped pairs,
    exported in one call and imported into a fresh pool in one call.  The
    restored rows of a stratified sample equal the oracle's registers, every
    restored row's checksum equals the original's, and the batch GET equals
    the per-key GET on 1,000 ids."""
    from redisson_amd import _lib, devmem
    from redisson_amd.hyperloglog import GroupedHyperLogLog
    from test_gpu_hll import _c5_stratified_sample

    G, n = 1_000_000, 500_000_000
    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
    pool = GroupedHyperLogLog(engine, G)
    pool.add(k.keys_fixed(n, 16), g)
    g.free()
    k.free()
    data, offs = pool.exportRedis()
    assert offs.size == G + 1 and int(offs[-1]) == data.size
    lens = np.diff(offs.astype(np.int64))
    # ~500 registers each: every key still sparse, but for the odd one holding a register above 32
    assert lens.min() > 16 and (lens > 3000).sum() <= 8 and set(lens[lens > 3000].tolist()) <= {12304}
    pick = np.random.default_rng(4).choice(G, 1000, replace=False).astype(np.uint64)
    for i in pick.tolist():
        assert bytes(data[int(offs[i]):int(offs[i + 1])]) == _export1(L, pool.pool, i), i
    pool2 = GroupedHyperLogLog(engine, G)
    pool2.importRedis(np.arange(G, dtype=np.uint64), data, offs)
    sample = _c5_stratified_sample(G)
    ref = np.zeros((sample.size, 16384), np.uint8)
    orc.hll_add_gen_grouped_ids(ref, G, sample, 0x5EED0006, 0, n, max(1, min(16, os.cpu_count() or 1)))
    for s, gid in enumerate(sample.tolist()):
        assert np.array_equal(pool2.registers(gid), ref[s]), gid
    # every row: a per-row checksum on the device copies (the pools' registers as bytes)
    a = L.rsk_hll_device_registers(pool.pool)
    b = L.rsk_hll_device_registers(pool2.pool)
    chunk = 65536
    for lo in range(0, G, chunk):
        m = min(chunk, G - lo)
        x = np.zeros(m * 16384, np.uint8)
        y = np.zeros(m * 16384, np.uint8)
        _lib.check(L.rsk_memcpy(engine.ctx, x.ctypes.data, ctypes.c_void_p(a + lo * 16384), x.size, 1))
        _lib.check(L.rsk_memcpy(engine.ctx, y.ctypes.data, ctypes.c_void_p(b + lo * 16384), y.size, 1))
        assert np.array_equal(x, y), lo
    data2, offs2 = pool2.exportRedis()
    assert np.array_equal(offs2, offs) and np.array_equal(data2, data)
    pool.close()
    pool2.close()


def test_export_import_through_registered_host_buffers(L, engine, orc):
    """rsk_host_register: the batched export / import DMA straight into / out of
    a caller-registered buffer (no pinned stage, no host copy) and give the same
    bytes and registers as the staged path; overlapping registrations and
    unregistering an unknown pointer are refused."""
    from redisson_amd import _lib, devmem
    from redisson_amd.hyperloglog import GroupedHyperLogLog

    G, n = 3000, 3_000_000
    g, k = devmem.gen_grouped(engine, 0x5EED0006, G, 0, n)
    pool = GroupedHyperLogLog(engine, G)
    pool.add(k.keys_fixed(n, 16), g)
    pool.mergeWith(np.arange(0, 300, dtype=np.uint64), np.arange(300, 600, dtype=np.uint64))  # some dense keys
    g.free()
    k.free()
    ids = np.arange(G, dtype=np.uint64)
    staged, offs = pool.exportRedis(ids)
    reg = np.zeros(staged.size + 4096, np.uint8)  # registered, larger than needed
    engine.host_register(reg)
    try:
        with pytest.raises(_lib.IllegalArgumentException):
            _lib.check(L.rsk_host_register(engine.ctx, reg.ctypes.data + 4096, 4096))  # overlaps
        data, offs2 = pool.exportRedis(ids, out=reg)
        assert np.array_equal(offs2, offs) and np.array_equal(reg[:staged.size], staged)
        fresh = GroupedHyperLogLog(engine, G)
        fresh.importRedis(ids, reg[:staged.size], offs)
        back, offs3 = fresh.exportRedis(ids)
        assert np.array_equal(offs3, offs) and np.array_equal(back, staged)
        for gid in (0, 299, 300, G - 1):
            assert np.array_equal(fresh.registers(gid), pool.registers(gid))
        fresh.close()
    finally:
        engine.host_unregister(reg)
    with pytest.raises(_lib.IllegalArgumentException):
        engine.host_unregister(reg)
    pool.close()


def test_export_on_every_copy_engine_gives_the_same_bytes(L, engine, orc, route):
    """The batched export's device->host copies on an SDMA engine chosen by
    measurement (route io_engine = 0), on each engine forced (io_engine = k:
    engine k - 1), and on HIP's copies (-1) give the same strings, staged
    through the pinned ring (io_pin = -1), into a buffer the call pins, and
    into a caller-registered buffer; the batched import's host->device copies
    on each of the same choices (and straight from a registered buffer) give
    the same registers; the measured engine is the fastest each way."""
    from redisson_amd import _lib

    rng = np.random.default_rng(31)
    G = 4000  # 49 MB of dense strings: several 16 MiB pieces
    rows = rng.integers(0, 25, size=(16, 16384), dtype=np.uint8)
    strs16 = [bytes(orc.hll_encode_dense(r)) for r in rows]
    pick = rng.integers(0, 16, G)
    strs = [strs16[j] for j in pick]
    want = np.frombuffer(b"".join(strs), np.uint8)
    h = _pool(L, engine, G)
    ids = np.arange(G)
    assert _import_batch(L, h, ids, strs) == 0
    route(io_engine=-1, io_pin=-1)
    rc, out, offs = _export_batch(L, h, ids)
    assert rc == 0 and np.array_equal(out[: want.size], want)
    route(io_engine=0, io_pin=-1)
    rc, out, offs = _export_batch(L, h, ids)
    assert rc == 0 and np.array_equal(out[: want.size], want)
    eng, rates = engine.copy_engine()
    assert eng >= 0, (eng, rates)
    assert rates[eng] == max(rates) > 0, rates
    for k in [e + 1 for e in range(8) if rates[e] > 0]:
        for pin in (-1, 0):  # (0 with a 256 MiB buffer: the call pins it)
            route(io_engine=k, io_pin=pin)
            rc, out, offs = _export_batch(L, h, ids, cap=None if pin else 256 << 20)
            assert rc == 0 and np.array_equal(out[: want.size], want), (k, pin)
    # the import's host->device copies: measured engine, each engine forced, HIP's copies
    ein, irates = engine.copy_engine(to_host=False)
    assert ein >= 0 and irates[ein] == max(irates) > 0, (ein, irates)
    for k in [0, -1] + [e + 1 for e in range(8) if irates[e] > 0]:
        route(io_engine=k)
        h2 = _pool(L, engine, G)
        assert _import_batch(L, h2, ids, strs) == 0, k
        route(io_engine=-1)
        rc, out, offs = _export_batch(L, h2, ids)
        assert rc == 0 and np.array_equal(out[: want.size], want), k
        for i in (0, 1, G // 2, G - 1):
            assert np.array_equal(_regs(L, h2, i), rows[pick[i]]), (k, i)
        L.rsk_hll_destroy(h2)
    route(io_engine=0, io_pin=0)
    reg = np.zeros(want.size + 8192, np.uint8)
    engine.host_register(reg)
    try:
        offs = np.zeros(G + 1, np.uint64)
        uids = ids.astype(np.uint64)
        _lib.check(L.rsk_hll_export_redis_batch(h, uids.ctypes.data, G, reg.ctypes.data, reg.size, offs.ctypes.data))
        assert int(offs[-1]) == want.size and np.array_equal(reg[: want.size], want)
        # and SET straight from the registered buffer (the engine reads it at its device address)
        h3 = _pool(L, engine, G)
        _lib.check(L.rsk_hll_import_redis_batch(h3, uids.ctypes.data, G, reg.ctypes.data, offs.ctypes.data))
        for i in (0, 1, G // 2, G - 1):
            assert np.array_equal(_regs(L, h3, i), rows[pick[i]]), i
        L.rsk_hll_destroy(h3)
    finally:
        engine.host_unregister(reg)
    L.rsk_hll_destroy(h)
