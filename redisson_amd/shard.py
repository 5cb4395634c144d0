"""Multi-GPU sharding: one process per GPU, the key stream split into
contiguous ranges, full sketches per GPU, and one merge step through the
RCCL layer of librsketch (rsk_comm.hip):

  HLL   : rsk_hll_allreduce        ncclAllReduce(uint8, MAX), 16 KiB
  pools : rsk_hll_allreduce_pool   the same over [n][16384]
          rsk_hll_reducescatter_pool  MAX reduce-scatter: rank r owns 1/N of the sketches (C5)
          rsk_hll_add_grouped_routed  pairs hashed where they live, 8-byte records
                                      sent to the rank owning their sketch (C5)
  Bloom : rsk_bloom_allreduce_or   slices to their owners, local OR, merged slices back

torch.distributed is used only as the out-of-band channel that ships the
RCCL unique id (any backend; gloo keeps the GPU out of torch's hands).  The
*_cpu functions restate the same exchange plans with torch.distributed on CPU
tensors so that the N > 1 logic is testable without GPUs (tests/test_shard_gloo.py).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass(frozen=True)
class ShardPlan:
    """Contiguous range partition of n keys over world ranks (weak scaling
    benches give every rank its own n instead)."""

    n: int
    world: int

    def range(self, rank: int):
        base, extra = divmod(self.n, self.world)
        start = rank * base + min(rank, extra)
        return start, start + base + (1 if rank < extra else 0)


def slice_words(nwords: int, nranks: int) -> int:
    """Words per rank in the Bloom slice-OR (a multiple of 4; N*S >= nwords).
    Mirrors rsk_bloom_allreduce_or."""
    s = (nwords + nranks - 1) // nranks
    return (s + 3) & ~3


def init_comm(engine, group=None) -> None:
    """Create the RCCL communicator of this rank (torch.distributed must be
    initialised; rank 0 creates the id, everyone else receives it)."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    if rank == 0:
        _lib.check(L.rsk_comm_unique_id(uid))
    box = [bytes(uid)]
    dist.broadcast_object_list(box, src=0, group=group)
    uid = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
    _lib.check(L.rsk_comm_init(engine.ctx, world, rank, uid), "rsk_comm_init")


def comm_info(engine):
    """(nranks, rank) as RCCL itself reports them for this context's
    communicator (ncclCommCount / ncclCommUserRank); (1, 0) without one."""
    n, r = ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.load().rsk_comm_info(engine.ctx, ctypes.byref(n), ctypes.byref(r)), "rsk_comm_info")
    return n.value, r.value


def hll_allreduce(pool, sketch_id: int = 0) -> None:
    _lib.check(_lib.load().rsk_hll_allreduce(pool, sketch_id), "rsk_hll_allreduce")


def hll_allreduce_pool(pool) -> None:
    _lib.check(_lib.load().rsk_hll_allreduce_pool(pool), "rsk_hll_allreduce_pool")


def owned_range(n: int, world: int, rank: int):
    """Sketches a rank owns after rsk_hll_reducescatter_pool: [r*q, (r+1)*q),
    q = n // world, plus the n % world tail on the last rank."""
    q = n // world
    return rank * q, q + (n - q * world if rank == world - 1 else 0)


def hll_reducescatter_pool(pool):
    """RCCL reduce-scatter (MAX) of a grouped pool; returns (first, count) of
    the sketches this rank now holds fully merged."""
    first, count = ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(_lib.load().rsk_hll_reducescatter_pool(pool, ctypes.byref(first), ctypes.byref(count)),
               "rsk_hll_reducescatter_pool")
    return first.value, count.value


def owner_of(ids, n: int, world: int) -> np.ndarray:
    """Rank owning each sketch id after the reduce-scatter (owned_range)."""
    q = n // world
    ids = np.asarray(ids, dtype=np.uint64)
    if q == 0:
        return np.full(ids.shape, world - 1, dtype=np.int64)
    return np.minimum(ids // np.uint64(q), np.uint64(world - 1)).astype(np.int64)


def hll_add_grouped_routed(pool, keys, groups, flags: int = 0):
    """Collective grouped PFADD routed to the owners (rsk_hll_add_grouped_routed):
    every rank passes its own device-resident 16-byte keys (a KeyBatch) and
    uint32 group ids (a DeviceBuffer); returns (first, count) of the sketches
    this rank owns, which then hold every rank's pairs."""
    first, count = ctypes.c_uint64(), ctypes.c_uint64()
    ks = keys.as_struct()
    _lib.check(_lib.load().rsk_hll_add_grouped_routed(pool, ctypes.byref(ks), groups.ptr if keys.n else None, flags,
                                                      ctypes.byref(first), ctypes.byref(count)),
               "rsk_hll_add_grouped_routed")
    return first.value, count.value


def route_plan(groups, n: int, world: int):
    """The routing plan of rsk_hll_add_grouped_routed restated: for each pair
    its owner (ids >= n dropped: -1) and its id local to the owner's range,
    and the pairs sent to each rank (records[o] in the send buffer are the
    pairs with owner o, in any order: MAX does not care)."""
    g = np.asarray(groups, dtype=np.uint64)
    valid = g < np.uint64(n)
    owner = np.where(valid, owner_of(np.where(valid, g, 0), n, world), -1)
    q = n // world
    local = np.where(valid, g - owner.clip(0).astype(np.uint64) * np.uint64(q), 0).astype(np.uint64)
    counts = np.bincount(owner[valid], minlength=world).astype(np.uint64)
    return owner, local, counts


def hll_add_grouped_routed_cpu(records, groups, n: int, group=None, heavy_min: int = 0, stats=None):
    """The routed grouped add on CPU tensors, same plan as the GPU path:
    `records` (uint32 index << 6 | rank per pair, the hash taken where the
    pair lives) and `groups` of this rank's pairs; pairs sorted by owner, the
    per-owner counts then the 8-byte records {local id, record} exchanged
    all-to-all, each rank maxing what it receives into its owned rows.
    heavy_min > 0: groups with at least that many pairs here that another rank
    owns are first folded into one local row each, and the rows (16384 bytes +
    a 4-byte id) travel instead of their records (rsk_comm.hip; the device
    takes the counts from a sample, this restatement the exact ones); the owner
    maxes them into its rows.  stats (a dict) gets the bytes this rank
    received.  Returns (first, count, owned rows [count][16384])."""
    import torch
    import torch.distributed as dist

    N, r = dist.get_world_size(group), dist.get_rank(group)
    owner, local, counts = route_plan(groups, n, N)
    g = np.asarray(groups, dtype=np.uint64)
    recs = np.asarray(records, np.uint32)
    heavy = np.zeros(g.shape, bool)
    hids = np.zeros(0, np.uint64)
    if heavy_min > 0:
        valid = owner >= 0
        ids, cnt = np.unique(g[valid], return_counts=True)
        hids = ids[(cnt >= heavy_min) & (owner_of(ids, n, N) != r)]  # ascending: each owner's rows contiguous
        heavy = valid & np.isin(g, hids)
    light = (owner >= 0) & ~heavy
    lcounts = np.bincount(owner[light], minlength=N).astype(np.int64)
    order = np.argsort(owner, kind="stable")
    order = order[light[order]]
    send = np.stack([local[order].astype(np.int64), recs[order].astype(np.int64)], 1)
    # heavy rows, folded here, and their ids (global), grouped by owner
    hrows = np.zeros((hids.size, 16384), np.uint8)
    if hids.size:
        slot = np.searchsorted(hids, g[heavy])
        rc = recs[heavy]
        np.maximum.at(hrows, (slot, (rc >> 6).astype(np.int64)), (rc & 63).astype(np.uint8))
    hcounts = np.bincount(owner_of(hids, n, N), minlength=N).astype(np.int64) if hids.size else np.zeros(N, np.int64)
    cin = torch.zeros(2 * N, dtype=torch.int64)
    dist.all_to_all_single(cin, torch.from_numpy(np.stack([lcounts, hcounts], 1).reshape(-1).copy()), group=group)
    cin = cin.numpy().reshape(N, 2)
    si, so = [int(x) for x in cin[:, 0]], [int(x) for x in lcounts]
    recv = torch.zeros(sum(si) * 2, dtype=torch.int64)
    dist.all_to_all_single(recv, torch.from_numpy(send.reshape(-1).copy()), output_split_sizes=[2 * x for x in si],
                           input_split_sizes=[2 * x for x in so], group=group)
    rec = recv.numpy().reshape(-1, 2)
    hi_, ho = [int(x) for x in cin[:, 1]], [int(x) for x in hcounts]
    rid = torch.zeros(sum(hi_), dtype=torch.int64)
    dist.all_to_all_single(rid, torch.from_numpy(hids.astype(np.int64)), output_split_sizes=hi_,
                           input_split_sizes=ho, group=group)
    rrows = torch.zeros(sum(hi_) * 16384, dtype=torch.uint8)
    dist.all_to_all_single(rrows, torch.from_numpy(hrows.reshape(-1).copy()), output_split_sizes=[16384 * x for x in hi_],
                           input_split_sizes=[16384 * x for x in ho], group=group)
    first, count = owned_range(n, N, r)
    rows = np.zeros((count, 16384), np.uint8)
    if rec.size:
        idx, rank = (rec[:, 1] >> 6).astype(np.int64), (rec[:, 1] & 63).astype(np.uint8)
        np.maximum.at(rows, (rec[:, 0], idx), rank)
    rr = rrows.numpy().reshape(-1, 16384)
    for gid, row in zip(rid.numpy(), rr):
        np.maximum(rows[int(gid) - first], row, out=rows[int(gid) - first])
    if stats is not None:
        own_light = int(lcounts[r])
        stats["recv_bytes"] = 8 * (int(sum(si)) - own_light) + (16384 + 4) * int(sum(hi_))
        stats["recv_rows"] = int(sum(hi_))
    return first, count, rows


def hll_fetch_rows(pool, ids, flags: int = 0) -> None:
    """Collective: make the local rows `ids` equal to their owners' rows
    (rsk_hll_fetch_rows), so countWith/mergeWith can read sketches owned by
    other ranks.  Every rank calls it, possibly with no ids.  flags =
    _lib.RSK_FETCH_SELF also routes owned ids through the exchange (tests)."""
    a = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64).ravel())
    _lib.check(_lib.load().rsk_hll_fetch_rows_flags(pool, a.ctypes.data if a.size else None, a.size, flags),
               "rsk_hll_fetch_rows")


def fetch_plan(n: int, world: int, rank: int, ids, flags: int = 0):
    """The request plan of rsk_hll_fetch_rows restated: (distinct ids asked of
    other ranks ascending, rows asked of each rank).  The library's own C++
    plan (rsk_plan_fetch) is checked against this in tests/test_plan.py."""
    want = np.unique(np.asarray(ids, dtype=np.uint64).ravel())
    assert want.size == 0 or int(want[-1]) < n
    if not flags & _lib.RSK_FETCH_SELF:
        want = want[owner_of(want, n, world) != rank]
    return want, np.bincount(owner_of(want, n, world), minlength=world).astype(np.uint64)


def bloom_allreduce_or(bloom, flags: int = 0) -> None:
    """Collective: the filter := OR over ranks (flags = _lib.RSK_FETCH_SELF also
    sends this rank's own slice through RCCL, so every step runs at N = 1)."""
    _lib.check(_lib.load().rsk_bloom_allreduce_or_flags(bloom, flags), "rsk_bloom_allreduce_or")


def init_comm_single(engine) -> None:
    """A 1-rank RCCL communicator without torch.distributed (N = 1 runs of the
    multi-GPU code path)."""
    L = _lib.load()
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(engine.ctx, 1, 0, uid), "rsk_comm_init")


# ------------------------------------------------------- CPU restatements
def hll_allreduce_cpu(regs: np.ndarray, group=None) -> np.ndarray:
    """The HLL exchange on CPU tensors: register-wise MAX over ranks."""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(regs, dtype=np.uint8).copy())
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.numpy()


def hll_reducescatter_pool_cpu(regs: np.ndarray, group=None):
    """The C5 exchange plan on CPU tensors: rank r receives the MAX over ranks
    of its owned rows (owned_range); returns (first, count, owned rows).  The
    tail rows go through an all-reduce, as in rsk_hll_reducescatter_pool."""
    import torch
    import torch.distributed as dist

    N, r = dist.get_world_size(group), dist.get_rank(group)
    G = regs.shape[0]
    q = G // N
    first, count = owned_range(G, N, r)
    out = np.empty((count, regs.shape[1]), np.uint8)
    if q:
        # reduce-scatter restated as N reductions of one slice each (gloo has no uint8 reduce_scatter)
        for j in range(N):
            t = torch.from_numpy(np.ascontiguousarray(regs[j * q:(j + 1) * q]).copy())
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            if j == r:
                out[:q] = t.numpy()
    if G - q * N:
        t = torch.from_numpy(np.ascontiguousarray(regs[q * N:]).copy())
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        if r == N - 1:
            out[q:] = t.numpy()
    return first, count, out


def hll_fetch_rows_cpu(regs: np.ndarray, ids, group=None) -> np.ndarray:
    """rsk_hll_fetch_rows restated on CPU tensors with the same plan: distinct
    non-owned ids grouped by owner in ascending order, counts then ids
    exchanged all-to-all, owners gather the rows in request order, rows sent
    back and written into the local pool `regs` ([G][16384], updated in place)."""
    import torch
    import torch.distributed as dist

    N, r = dist.get_world_size(group), dist.get_rank(group)
    G, R = regs.shape
    want, cnt_out = fetch_plan(G, N, r, ids)  # sorted by id, hence grouped by owner
    cnt_out = cnt_out.astype(np.int64)
    cnt_in = torch.zeros(N, dtype=torch.int64)
    dist.all_to_all_single(cnt_in, torch.from_numpy(cnt_out.copy()), group=group)
    cnt_in = cnt_in.numpy()
    so, si = [int(x) for x in cnt_out], [int(x) for x in cnt_in]
    asked = torch.zeros(int(cnt_in.sum()), dtype=torch.int64)
    dist.all_to_all_single(asked, torch.from_numpy(want.astype(np.int64)), output_split_sizes=si,
                           input_split_sizes=so, group=group)
    rows_send = torch.from_numpy(np.ascontiguousarray(regs[asked.numpy().astype(np.uint64)]).reshape(-1))
    rows_recv = torch.zeros(want.size * R, dtype=torch.uint8)
    dist.all_to_all_single(rows_recv, rows_send, output_split_sizes=[x * R for x in so],
                           input_split_sizes=[x * R for x in si], group=group)
    if want.size:
        regs[want] = rows_recv.numpy().reshape(want.size, R)
    return regs


def bloom_slice_bounds(nwords: int, world: int, rank: int):
    """Words [lo, hi) of the filter rank `rank` merges (rsk_bloom_allreduce_or:
    slices of slice_words() words, the last ones short or empty)."""
    S = slice_words(nwords, world)
    lo = min(rank * S, nwords)
    return lo, min(lo + S, nwords)


def bloom_allreduce_or_cpu(bits: np.ndarray, group=None) -> np.ndarray:
    """The Bloom slice-OR exchange on CPU tensors, same plan as the GPU path:
    phase 1 sends slice j of every rank to rank j (ragged slices, nothing
    padded), rank j ORs them into its own slice, phase 2 sends the merged
    slice back to every rank."""
    import torch
    import torch.distributed as dist

    N, r = dist.get_world_size(group), dist.get_rank(group)
    nbytes = bits.size
    nwords = ((nbytes + 15) // 16) * 4
    words = np.zeros(nwords * 4, np.uint8)
    words[:nbytes] = bits
    words = words.view(np.uint32)
    bounds = [bloom_slice_bounds(nwords, N, j) for j in range(N)]
    sizes = [hi - lo for lo, hi in bounds]
    lo, hi = bounds[r]
    recv = torch.zeros(N * sizes[r], dtype=torch.int32)
    dist.all_to_all_single(recv, torch.from_numpy(words.view(np.int32).copy()),
                           output_split_sizes=[sizes[r]] * N, input_split_sizes=sizes, group=group)
    rows = recv.numpy().view(np.uint32).reshape(N, sizes[r])
    merged = words.copy()
    merged[lo:hi] = np.bitwise_or.reduce(rows, axis=0) if sizes[r] else merged[lo:hi]
    back = torch.zeros(nwords, dtype=torch.int32)
    dist.all_to_all_single(back, torch.from_numpy(np.tile(merged[lo:hi].view(np.int32), N)),
                           output_split_sizes=sizes, input_split_sizes=[sizes[r]] * N, group=group)
    return back.numpy().view(np.uint8)[:nbytes].copy()
