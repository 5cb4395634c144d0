"""The routed grouped add (rsk_hll_add_grouped_routed) at the C5 per-GPU size
on one GPU through the self exchange (every record and heavy row through RCCL
to itself), uniform or Zipf groups, with route overrides (route_heavy=-1: no
pre-combine).  Wall time per call and per-stage HIP-event times, one JSON line.

  python scripts/routed_profile.py [reps] [zipf_s|0] [route=value,...]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem, shard  # noqa: E402
from redisson_amd.hyperloglog import GroupedHyperLogLog  # noqa: E402

STAGES = ("hll_route", "hll_route_heavy", "hll_route_heavy_rows", "hll_route_counts", "hll_route_exchange",
          "hll_gpart1", "hll_gpart2", "hll_gapply", "hll_route_rows_merge")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    zipf = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    routes = dict(kv.split("=") for kv in sys.argv[3].split(",")) if len(sys.argv) > 3 and sys.argv[3] else {}
    L = _lib.load()
    _lib.diag()
    eng = _lib.Engine(0)
    for k, v in routes.items():
        eng.set_route(k, int(v))
    uid = (ctypes.c_uint8 * 128)()
    _lib.check(L.rsk_comm_unique_id(uid))
    _lib.check(L.rsk_comm_init(eng.ctx, 1, 0, uid))
    G, n = 1_000_000, 500_000_000
    if zipf:
        g, k = devmem.gen_grouped_zipf(eng, 0x5EED0006, G, zipf, 0, n)
    else:
        g, k = devmem.gen_grouped(eng, 0x5EED0006, G, 0, n)
    kb = k.keys_fixed(n, 16)
    pool = GroupedHyperLogLog(eng, G)
    pool.clear()
    shard.hll_add_grouped_routed(pool.pool, kb, g, flags=_lib.RSK_FETCH_SELF)  # warm-up (buffers)
    eng.sync()
    eng.prof_reset()
    eng.prof_enable(True)
    ts = []
    for _ in range(reps):
        pool.clear()
        t0 = time.perf_counter()
        shard.hll_add_grouped_routed(pool.pool, kb, g, flags=_lib.RSK_FETCH_SELF)
        ts.append(time.perf_counter() - t0)
    eng.prof_enable(False)
    st = {}
    for s in STAGES:
        ms, cnt = eng.prof_read(s)
        if cnt:
            st[s] = ms / reps
    print(json.dumps({"routes": routes, "zipf": zipf, "reps": reps, "call_ms": min(ts) * 1e3,
                      "call_ms_each": [t * 1e3 for t in ts], "stage_ms_per_call": st}), flush=True)
    _lib.check(L.rsk_comm_destroy(eng.ctx))


if __name__ == "__main__":
    main()
