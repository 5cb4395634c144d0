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
