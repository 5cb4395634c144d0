"""Partitioned Bloom add at C3 size under tuning knobs (env read per call):
per-stage device times for each configuration, and the bit count as a check.

    python scripts/bloom_part_tune.py OUT.json [n] [CONFIG ...]

CONFIG = "RSK_BLOOM_G_PER_CU=2,RSK_BLOOM_P2_PER_CU=4" (comma-separated env
assignments); "RSK_BLOOM_PARTITION=0" times the direct atomicOr kernel."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402

if os.environ.get("RSK_TUNE_TORCH"):  # A/B: the bench process also imports torch
    _lib.load()
    import torch  # noqa: F401

STAGES = ("bloom_part_hist", "bloom_part1", "bloom_part2", "bloom_slice_apply", "bloom_st1", "bloom_st_mid",
          "bloom_st2", "bloom_st_apply", "bloom_add16")


def main():
    out_path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
    configs = sys.argv[3:] or [""]
    L = _lib.load()
    eng = _lib.Engine(0)
    size = ctypes.c_int64()
    k = ctypes.c_int32()
    _lib.check(L.rsk_bloom_params(n, 0.01, _lib.RSK_BLOOM_EXTENDED, ctypes.byref(size), ctypes.byref(k)))
    ins = devmem.gen_keys16(eng, 0x5EED0003, 0, n)
    extra = []
    if os.environ.get("RSK_TUNE_QBUF"):  # A/B: the bench also holds the 1B query keys
        extra.append(devmem.gen_keys16(eng, 0x5EED0004, 0, n))
    ks = ins.keys_fixed(n, 16).as_struct()
    res = {"n": n, "size": size.value, "k": k.value, "configs": {}}
    for cfg in configs:
        env = dict(kv.split("=") for kv in cfg.split(",") if kv)
        saved = {key: os.environ.get(key) for key in env}
        os.environ.update(env)
        row = {}
        for rep in range(3):
            b = ctypes.c_void_p()
            _lib.check(L.rsk_bloom_create(eng.ctx, size.value, k.value, ctypes.byref(b)))
            eng.prof_reset()
            eng.prof_enable(rep > 0)
            _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
            eng.sync()
            eng.prof_enable(False)
            bc = ctypes.c_uint64()
            _lib.check(L.rsk_bloom_bitcount(b, ctypes.byref(bc)))
            L.rsk_bloom_destroy(b)
            if rep:
                for s in STAGES:
                    ms, cnt = eng.prof_read(s)
                    if cnt:
                        row.setdefault(s, []).append(ms)
                row.setdefault("bitcount", []).append(bc.value)
        for key, v in saved.items():
            if v is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = v
        summary = {s: min(v) for s, v in row.items() if s != "bitcount"}
        summary["bitcount"] = row["bitcount"][0]
        res["configs"][cfg or "default"] = summary
        print(cfg or "default", json.dumps(summary), flush=True)
    ins.free()
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
