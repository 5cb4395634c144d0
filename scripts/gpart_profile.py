"""Grouped PFADD (BASELINE C5, per GPU) alone in a process: per-stage HIP-event
times of rsk_hll_add_grouped over 500M pairs into 1M sketches, with optional
route overrides (A/B of kernel forms, interleaved by the caller).

  python scripts/gpart_profile.py [reps] [zipf_s|0] [route=value,...]   -> one JSON line"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402
from redisson_amd.hyperloglog import GroupedHyperLogLog  # noqa: E402

STAGES = ("hll_gpart_count", "hll_gpart1", "hll_gpart2", "hll_gapply", "hll_add_grouped16")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    zipf = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    routes = dict(kv.split("=") for kv in sys.argv[3].split(",")) if len(sys.argv) > 3 else {}
    _lib.load()
    _lib.diag()
    eng = _lib.Engine(0)
    for k, v in routes.items():
        eng.set_route(k, int(v))
    G, n = 1_000_000, 500_000_000
    if zipf:
        groups, keys = devmem.gen_grouped_zipf(eng, 0x5EED0006, G, zipf, 0, n)
    else:
        groups, keys = devmem.gen_grouped(eng, 0x5EED0006, G, 0, n)
    kb = keys.keys_fixed(n, 16)
    pool = GroupedHyperLogLog(eng, G)
    pool.add(kb, groups)  # warm-up (scratch)
    eng.sync()
    eng.prof_reset()
    eng.prof_enable(True)
    for _ in range(reps):
        pool.clear()
        pool.add(kb, groups)
    eng.sync()
    eng.prof_enable(False)
    st = {}
    for s in STAGES:
        ms, cnt = eng.prof_read(s)
        if cnt:
            st[s] = ms / reps
    print(json.dumps({"routes": routes, "zipf": zipf, "reps": reps, "stage_ms": st,
                      "add_ms": sum(st.values())}), flush=True)


if __name__ == "__main__":
    main()
