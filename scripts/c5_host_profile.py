"""Wall time of each call of the C5 step (clear, grouped add, count of all
sketches, 10^5 countWith, 10^5 mergeWith) next to the GPU time the library's
HIP events give for the same calls: the difference is host work.
python scripts/c5_host_profile.py [pairs] [groups] [steps]   -> one JSON line"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402
from redisson_amd.hyperloglog import GroupedHyperLogLog  # noqa: E402

KERNELS = ("hll_clear", "hll_gpart_count", "hll_gpart1", "hll_gpart2", "hll_gapply", "hll_count", "hll_union_count",
           "hll_merge")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000_000
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    eng = _lib.Engine(0)
    groups, keys = devmem.gen_grouped(eng, 0x5EED0007, G, 0, n)
    kb = keys.keys_fixed(n, 16)
    pool = GroupedHyperLogLog(eng, G)
    rng = np.random.default_rng(5)
    ops = 100_000
    cw = np.stack([rng.integers(0, G, ops, dtype=np.uint64), rng.integers(0, G, ops, dtype=np.uint64)], 1)
    md, ms = rng.integers(0, G, ops, dtype=np.uint64), rng.integers(0, G, ops, dtype=np.uint64)
    calls = {"clear": lambda: pool.clear(), "add": lambda: pool.add(kb, groups), "count_all": lambda: pool.count(),
             "countWith": lambda: pool.countWith(cw), "mergeWith": lambda: pool.mergeWith(md, ms)}
    wall = {k: [] for k in calls}
    for s in range(steps + 2):
        if s == 2:
            eng.prof_reset()
            eng.prof_enable(True)
        for name, fn in calls.items():
            eng.sync()
            t0 = time.perf_counter()
            fn()
            eng.sync()
            if s >= 2:
                wall[name].append((time.perf_counter() - t0) * 1e3)
    eng.prof_enable(False)
    gpu = {k: eng.prof_read(k)[0] / steps for k in KERNELS}
    print(json.dumps({"pairs": n, "groups": G, "steps": steps,
                      "wall_ms_median": {k: float(np.median(v)) for k, v in wall.items()},
                      "gpu_ms_per_step": gpu}))


if __name__ == "__main__":
    main()
