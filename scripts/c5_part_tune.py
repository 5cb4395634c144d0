"""Partitioned grouped PFADD (C5 size) under tuning knobs (env read per call):
per-stage device times per configuration, best of 3, on a cleared pool.

    python scripts/c5_part_tune.py OUT.json [n] [G] [CONFIG ...]

CONFIG = "RSK_HLL_GPART_G=2,RSK_HLL_GPART_GU=8" (comma-separated env assignments)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402

STAGES = ("hll_gpart_count", "hll_gpart1", "hll_gpart2", "hll_gapply")


def main():
    out_path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 500_000_000
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
    configs = sys.argv[4:] or [""]
    L = _lib.load()
    eng = _lib.Engine(0)
    groups, keys = devmem.gen_grouped(eng, 0x5EED0006, G, 0, n)
    ks = keys.keys_fixed(n, 16).as_struct()
    h = ctypes.c_void_p()
    _lib.check(L.rsk_hll_create(eng.ctx, G, ctypes.byref(h)))
    res = {"n": n, "G": G, "configs": {}}
    for cfg in configs:
        env = dict(kv.split("=") for kv in cfg.split(",") if kv)
        saved = {key: os.environ.get(key) for key in env}
        os.environ.update(env)
        best = None
        for _ in range(3):
            _lib.check(L.rsk_hll_clear(h))
            eng.prof_reset()
            eng.prof_enable(True)
            _lib.check(L.rsk_hll_add_grouped(h, ctypes.byref(ks), groups.ptr))
            eng.sync()
            eng.prof_enable(False)
            row = {st: eng.prof_read(st)[0] for st in STAGES}
            row["total"] = sum(row[st] for st in STAGES)
            if best is None or row["total"] < best["total"]:
                best = row
        cnt = (ctypes.c_uint64 * 4)()
        ids = (ctypes.c_uint64 * 4)(0, 1, G // 2, G - 1)
        _lib.check(L.rsk_hll_count(h, ids, 4, cnt))
        best["counts"] = list(cnt)
        res["configs"][cfg or "default"] = best
        print(cfg or "default", json.dumps(best), flush=True)
        for key, v in saved.items():
            if v is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = v
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
