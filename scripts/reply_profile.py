"""RBloomFilter.add() with replies at the C3 size, alone in a process (for
rocprofv3 kernel traces and PMC passes of the reply pipeline without the
reply-less insert's kernels of the same names):
1B keys (the C3 insert stream) into a fresh 1%-FPP EXTENDED filter, one
warm-up call (scratch allocation) and RUNS timed calls with per-stage HIP-event
times.   python scripts/reply_profile.py [n] [runs]   -> one JSON line"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402

STAGES = ("bloom_rp1", "bloom_rp_mid", "bloom_rp2", "bloom_rp_apply", "bloom_rp_reply", "bloom_rp_fallback")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    routes = dict(kv.split("=") for kv in sys.argv[3].split(",")) if len(sys.argv) > 3 else {}
    L = _lib.load()
    if routes:
        _lib.diag()
    eng = _lib.Engine(0)
    for name, v in routes.items():
        eng.set_route(name, int(v))
    size, k = ctypes.c_int64(), ctypes.c_int32()
    _lib.check(L.rsk_bloom_params(n, 0.01, _lib.RSK_BLOOM_EXTENDED, ctypes.byref(size), ctypes.byref(k)))
    keys = devmem.gen_keys16(eng, 0x5EED0003, 0, n)
    ks = keys.keys_fixed(n, 16).as_struct()
    out = devmem.DeviceBuffer(eng, n)
    times = []
    for r in range(runs + 1):
        if r == 1:
            eng.prof_reset()
            eng.prof_enable(True)
        b = ctypes.c_void_p()
        _lib.check(L.rsk_bloom_create(eng.ctx, size.value, k.value, ctypes.byref(b)))
        eng.sync()
        t0 = time.perf_counter()
        _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), out.ptr))
        eng.sync()
        if r:
            times.append(time.perf_counter() - t0)
        L.rsk_bloom_destroy(b)
    eng.prof_enable(False)
    stages = {}
    for s in STAGES:
        ms, cnt = eng.prof_read(s)
        if cnt:
            stages[s] = ms / runs
    trues = int(out.to_numpy().sum())
    print(json.dumps({"routes": routes, "keys": n, "size_bits": size.value, "k": k.value, "runs": runs,
                      "ms_min": min(times) * 1e3, "ms_all": [t * 1e3 for t in times],
                      "keys_per_s": n / min(times), "stage_ms_per_call": stages, "replies_true": trues}))


if __name__ == "__main__":
    main()
