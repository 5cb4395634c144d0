"""Batched Redis export / import of the C5 pool (1M sketches after 500M
grouped pairs) alone in a process: wall time of each call and the device time
of its kernels (rsk_hll_export_redis_batch / rsk_hll_import_redis_batch).

  python scripts/io_profile.py [reps] [merges] [route=value,...]   -> one JSON line

merges: that many random mergeWith pairs after the add (the bench's C5 pool:
10^5, which leaves ~95k destinations dense -- half the checkpoint's bytes)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from redisson_amd import _lib, devmem  # noqa: E402
from redisson_amd.hyperloglog import GroupedHyperLogLog  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    merges = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    routes = dict(kv.split("=") for kv in sys.argv[3].split(",")) if len(sys.argv) > 3 and sys.argv[3] else {}
    _lib.load()
    _lib.diag()
    if os.environ.get("IO_TORCH"):  # (as bench.py: torch imported after the library)
        import torch.distributed  # noqa: F401
    eng = _lib.Engine(0)
    for k_, v_ in routes.items():
        eng.set_route(k_, int(v_))
    if os.environ.get("IO_TRACE"):
        eng.set_route("io_trace", 1)  # host phase times of each call to stderr
    G, n = 1_000_000, 500_000_000
    g, k = devmem.gen_grouped(eng, 0x5EED0006, G, 0, n)
    pool = GroupedHyperLogLog(eng, G)
    pool.add(k.keys_fixed(n, 16), g)
    g.free()
    k.free()
    if merges:
        rng = np.random.default_rng(5)
        pool.mergeWith(rng.integers(0, G, size=merges, dtype=np.uint64), rng.integers(0, G, size=merges, dtype=np.uint64))
    ids = np.arange(G, dtype=np.uint64)
    data, offs = pool.exportRedis(ids)
    thp = os.environ.get("IO_THP")
    if thp is not None:  # the output buffer from an anonymous mapping with (1) or without (0) MADV_HUGEPAGE
        import mmap

        mm = mmap.mmap(-1, (data.size + (2 << 20) - 1) // (2 << 20) * (2 << 20))
        mm.madvise(mmap.MADV_HUGEPAGE if thp == "1" else mmap.MADV_NOHUGEPAGE)
        buf = np.frombuffer(mm, np.uint8)
        buf[:] = 0  # touch (faults the pages in, huge where granted)
        data, offs = pool.exportRedis(ids, out=buf)
    fresh = GroupedHyperLogLog(eng, G)
    fresh.importRedis(ids, data, offs)
    eng.prof_reset()
    eng.prof_enable(True)
    te, ti = [], []
    no_import = bool(os.environ.get("IO_NOIMPORT"))  # (exports back to back)
    for _ in range(reps):
        t0 = time.perf_counter()
        pool.exportRedis(ids, out=data)
        te.append(time.perf_counter() - t0)
        if no_import:
            continue
        t0 = time.perf_counter()
        fresh.importRedis(ids, data, offs)
        ti.append(time.perf_counter() - t0)
    ti = ti or [float("nan")]
    eng.prof_enable(False)
    dev = {s: eng.prof_read(s)[0] / reps for s in ("hll_export_encode", "hll_export_pack", "hll_import_check",
                                                    "hll_import_write")}
    print(json.dumps({"routes": routes, "sketches": G, "merges": merges, "bytes": int(offs[-1]), "export_ms": min(te) * 1e3, "import_ms": min(ti) * 1e3,
                      "export_ms_each": [round(t * 1e3, 2) for t in te], "no_import": no_import,
                      "thp": os.environ.get("IO_THP"), "torch": bool(os.environ.get("IO_TORCH")),
                      "device_ms": dev}), flush=True)
    if os.environ.get("IO_SDMA"):  # per-engine copy rates in this same process (scripts/sdma_probe.cpp)
        import ctypes

        lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libsdma_probe.so"))
        lib.sdma_probe_run.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        lib.sdma_probe_run(64, 1, 4)


if __name__ == "__main__":
    main()
