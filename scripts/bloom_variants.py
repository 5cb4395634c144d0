"""Bloom contains kernel variants at C3 size: timing (interleaved rounds) and
identical-output check against variant 0.  python scripts/bloom_variants.py OUT.json"""
import ctypes
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402

NAMES = {0: "all_k-1_parallel", 1: "early_exit_U1_32wg", 2: "early_exit_U2_32wg", 3: "early_exit_U4_32wg",
         4: "early_exit_U1_8wg", 5: "early_exit_U2_8wg", 6: "phased_U2_P2", 7: "phased_U2_P3",
         8: "phased_U1_P3", 9: "phased_U1_P6", 10: "phased_U4_P2", 11: "phased_U1_P2"}


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "bloom_variants.json"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
    L = _lib.load()
    D = _lib.diag()
    eng = _lib.Engine(0)
    size = ctypes.c_int64()
    k = ctypes.c_int32()
    _lib.check(L.rsk_bloom_params(n, 0.01, _lib.RSK_BLOOM_EXTENDED, ctypes.byref(size), ctypes.byref(k)))
    b = ctypes.c_void_p()
    _lib.check(L.rsk_bloom_create(eng.ctx, size.value, k.value, ctypes.byref(b)))
    ins = devmem.gen_keys16(eng, 0x5EED0003, 0, n)
    ks = ins.keys_fixed(n, 16).as_struct()
    _lib.check(L.rsk_bloom_add(b, ctypes.byref(ks), None))
    ins.free()
    qs = devmem.gen_queries16(eng, 0x5EED0004, 0x5EED0003, n, 0, n)
    outs = {v: devmem.DeviceBuffer(eng, n) for v in NAMES}
    t = {v: [] for v in NAMES}
    for _ in range(4):
        for v in NAMES:
            ms = ctypes.c_double()
            _lib.check_diag(D.rsk_diag_bloom_contains_variant(eng.ctx, v, b, qs.ptr, n, outs[v].ptr, ctypes.byref(ms)))
            t[v].append(ms.value)
    ref = outs[0].to_numpy()
    res = {"n": n, "size": size.value, "k": k.value, "variants": {}}
    for v, nm in NAMES.items():
        same = bool(np.array_equal(outs[v].to_numpy(), ref)) if v else True
        med = statistics.median(t[v])
        res["variants"][nm] = {"median_ms": med, "min_ms": min(t[v]), "keys_per_s": n / med * 1e3, "identical": same}
        print("%-22s %8.2f ms  %.3g keys/s  identical=%s" % (nm, med, n / med * 1e3, same), flush=True)
    res["true_count"] = int(ref.sum())
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
