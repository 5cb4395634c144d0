"""The C++ exchange plans of the RCCL layer (rsk_plan.hip, called by
rsk_comm.hip) against redisson_amd/shard.py, whose restatement the gloo tests
(tests/test_shard_gloo.py) run end to end at world sizes 2 and 3.  Pure host
arithmetic: runs on CPU through the C ABI (no GPU call), at N = 1, 2, 3, 8 and
beyond, with pools smaller than N and with tails."""
import ctypes
import os

import numpy as np
import pytest

from redisson_amd import _lib, shard


class _PlanLib:
    """librsketch's exported plan functions, or (RSK_PLAN_LIB) the same
    source built alone under ASan/UBSan (oracle/Makefile `asan`)."""

    def __init__(self):
        path = os.environ.get("RSK_PLAN_LIB")
        if not path:
            self.L = _lib.load()
            return
        self.L = ctypes.CDLL(path)
        for name, (res, args) in _lib.SIGNATURES.items():
            if name.startswith("rsk_plan_"):
                fn = getattr(self.L, name)
                fn.restype, fn.argtypes = res, args

    def __getattr__(self, name):
        return getattr(self.L, name)


_PL = None


def plan_lib():
    global _PL
    if _PL is None:
        _PL = _PlanLib()
    return _PL


WORLDS = [1, 2, 3, 5, 8, 16]
POOLS = [1, 2, 3, 7, 8, 9, 20, 1000, 1000003]


def _ck(rc):
    if rc != _lib.RSK_OK:
        raise _lib.IllegalArgumentException("rsk_plan_* returned %d" % rc)


def _c_owned(n, N, r):
    f, c = ctypes.c_uint64(), ctypes.c_uint64()
    _ck(plan_lib().rsk_plan_owned_range(n, N, r, ctypes.byref(f), ctypes.byref(c)))
    return f.value, c.value


def _c_fetch(n, N, r, ids, flags=0):
    L = plan_lib()
    ids = np.ascontiguousarray(np.asarray(ids, np.uint64))
    want = np.zeros(max(1, ids.size), np.uint64)
    cnt = np.zeros(N, np.uint64)
    nw = ctypes.c_uint64()
    _ck(L.rsk_plan_fetch(n, N, r, ids.ctypes.data if ids.size else None, ids.size, flags,
                         want.ctypes.data, ctypes.byref(nw), cnt.ctypes.data))
    return want[:nw.value], cnt


@pytest.mark.parametrize("N", WORLDS)
def test_owned_ranges_match_shard_py_and_tile_the_pool(N):
    L = plan_lib()
    for n in POOLS:
        covered = 0
        for r in range(N):
            f, c = _c_owned(n, N, r)
            assert (f, c) == shard.owned_range(n, N, r)
            assert f == covered or c == 0
            covered = f + c if c else covered
        assert covered == n  # contiguous, disjoint, complete (G < N: all on the last rank)
        ids = np.unique(np.linspace(0, n - 1, num=min(n, 257)).astype(np.uint64))
        own_py = shard.owner_of(ids, n, N)
        for i, want in zip(ids, own_py):
            o = ctypes.c_int()
            _ck(L.rsk_plan_owner(n, N, int(i), ctypes.byref(o)))
            assert o.value == int(want)
            f, c = _c_owned(n, N, o.value)
            assert f <= int(i) < f + c


@pytest.mark.parametrize("N", WORLDS)
def test_shard_ranges_match_shardplan(N):
    L = plan_lib()
    for n in [0, 1, 5, 8, 1000, 10**9 + 7, 8 * 10**9]:
        end_prev = 0
        for r in range(N):
            b, e = ctypes.c_uint64(), ctypes.c_uint64()
            _ck(L.rsk_plan_shard_range(n, N, r, ctypes.byref(b), ctypes.byref(e)))
            assert (b.value, e.value) == shard.ShardPlan(n, N).range(r)
            assert b.value == end_prev
            end_prev = e.value
        assert end_prev == n


@pytest.mark.parametrize("N", WORLDS)
def test_bloom_slice_words_match(N):
    L = plan_lib()
    for nwords in [4, 8, 12, 1000, 299_533_076, 2**30 + 4]:
        s = ctypes.c_uint64()
        _ck(L.rsk_plan_bloom_slice_words(nwords, N, ctypes.byref(s)))
        assert s.value == shard.slice_words(nwords, N)
        assert s.value % 4 == 0 and s.value * N >= nwords


@pytest.mark.parametrize("N", WORLDS)
@pytest.mark.parametrize("flags", [0, _lib.RSK_FETCH_SELF])
def test_fetch_plan_matches_shard_py(N, flags):
    rng = np.random.default_rng(1000 + N + 7 * flags)
    for n in POOLS:
        for r in range(N):
            for m in [0, 1, 5, 300]:
                ids = rng.integers(0, n, size=m, dtype=np.uint64)
                if m:
                    ids = np.concatenate([ids, ids[:2]])  # duplicates are fetched once
                want_c, cnt_c = _c_fetch(n, N, r, ids, flags)
                want_p, cnt_p = shard.fetch_plan(n, N, r, ids, flags)
                assert np.array_equal(want_c, want_p)
                assert np.array_equal(cnt_c, cnt_p)
                # ascending ids are grouped by owner in rank order; counts sum to the request
                owners = shard.owner_of(want_c, n, N)
                assert np.all(np.diff(owners) >= 0)
                assert int(cnt_c.sum()) == want_c.size
                if not flags:
                    assert cnt_c[r] == 0


def test_fetch_plan_rejects_out_of_range_ids():
    bad = np.array([5, 20], np.uint64)
    with pytest.raises(_lib.IllegalArgumentException):
        _c_fetch(20, 2, 0, bad)


def test_plan_argument_checks():
    L = plan_lib()
    f, c = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.rsk_plan_owned_range(10, 0, 0, ctypes.byref(f), ctypes.byref(c)) == _lib.RSK_ERR_INVALID_ARG
    assert L.rsk_plan_owned_range(10, 2, 2, ctypes.byref(f), ctypes.byref(c)) == _lib.RSK_ERR_INVALID_ARG
    o = ctypes.c_int()
    assert L.rsk_plan_owner(10, 2, 10, ctypes.byref(o)) == _lib.RSK_ERR_INVALID_ARG


def _route_recv(counts, G, N, heavy_min, cap=65536):
    rb, rr, ap = (np.zeros(N, np.uint64) for _ in range(3))
    c = np.ascontiguousarray(counts, np.uint64)
    _ck(plan_lib().rsk_plan_route_recv(c.ctypes.data, G, N, heavy_min, cap, rb.ctypes.data, rr.ctypes.data,
                                       ap.ctypes.data))
    return rb, rr, ap


def test_route_plan_small_by_hand():
    # G = 6, N = 2 (rank 0 owns 0..2, rank 1 owns 3..5); heavy at >= 4 pairs
    counts = np.array([[5, 1, 0, 4, 2, 0],
                       [0, 4, 0, 9, 3, 1]], np.uint64)
    rb, rr, ap = _route_recv(counts, 6, 2, 4)
    # rank 0 receives from rank 1: group 1 (4 pairs, heavy: a row); rank 1 from rank 0: group 3 (a row), group 4 (2)
    assert rr.tolist() == [1, 1]
    assert rb.tolist() == [16388, 16388 + 16]
    # applied light records: rank 0 its own 5 + 1 (groups 0, 1 own), rank 1 own 9 + 3 + 1 and rank 0's 2 of group 4
    assert ap.tolist() == [6, 15]
    rb0, rr0, ap0 = _route_recv(counts, 6, 2, 0)  # no pre-combine
    assert rr0.tolist() == [0, 0] and rb0.tolist() == [8 * 4, 8 * 6] and ap0.tolist() == [10, 19]


def test_route_plan_zipf_balance_at_8_ranks():
    """VERDICT r05 Next 2 at the C5 configuration: N = 8, G = 1M, 5e8 pairs per
    rank drawn Zipf(1.1) (expected counts).  Contiguous ownership sends rank 0
    ~26 GB (7.4x a uniform rank's 3.5 GB); with groups of >= 2048 pairs owned
    elsewhere pre-combined into rows, rank 0 receives <= 1.25x the uniform
    per-rank bytes, and no rank more.  (The other ranks receive far less than
    uniform, so max/mean bytes stays ~5: the Zipf traffic itself lands in rank
    0's range; what bounds the step is the max.)"""
    G, N, n = 1_000_000, 8, 500_000_000
    w = np.arange(1, G + 1, dtype=np.float64) ** -1.1
    cz = np.rint(n * w / w.sum()).astype(np.uint64)
    cu = np.full(G, n // G, np.uint64)
    uni, _, uni_ap = _route_recv(np.tile(cu, (N, 1)), G, N, 2048)
    raw, _, raw_ap = _route_recv(np.tile(cz, (N, 1)), G, N, 0)
    pre, rows, pre_ap = _route_recv(np.tile(cz, (N, 1)), G, N, 2048)
    assert raw[0] > 7 * uni[0]
    assert pre[0] <= 1.25 * uni[0] and pre.max() == pre[0]
    assert rows[0] > 0 and rows[1:].sum() == 0
    assert int(pre_ap.sum()) < int(raw_ap.sum())  # heavy pairs folded at the source, not applied at the owner
