"""Wall time of each call in the C5 step (host overhead vs kernel time)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402
from redisson_amd.hyperloglog import GroupedHyperLogLog  # noqa: E402


def main():
    eng = _lib.Engine(0)
    G, n = 1_000_000, 500_000_000
    groups, keys = devmem.gen_grouped(eng, 0x5EED0006, G, 0, n)
    kb = keys.keys_fixed(n, 16)
    pool = GroupedHyperLogLog(eng, G)
    rng = np.random.default_rng(5)
    cw = rng.integers(0, G, size=(100_000, 2), dtype=np.uint64)
    md = rng.integers(0, G, size=100_000, dtype=np.uint64)
    ms_ = rng.integers(0, G, size=100_000, dtype=np.uint64)
    eng.prof_enable(True)
    for rep in range(3):
        t = [time.perf_counter()]
        pool.add(kb, groups)
        eng.sync()
        t.append(time.perf_counter())
        pool.count()
        t.append(time.perf_counter())
        pool.countWith(cw)
        t.append(time.perf_counter())
        pool.mergeWith(md, ms_)
        t.append(time.perf_counter())
        d = np.diff(t) * 1e3
        print("rep %d add %.2f count %.2f countWith %.2f mergeWith %.2f ms" % (rep, *d), flush=True)
    for k in ("hll_add_grouped16", "hll_count", "hll_union_count", "hll_merge"):
        ms, cnt = eng.prof_read(k)
        print(k, "%.3f ms/launch" % (ms / max(1, cnt)), cnt)


if __name__ == "__main__":
    main()
