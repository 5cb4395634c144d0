"""Roofline denominators and HLL kernel variants, measured on the GPU box.

python scripts/membench.py OUT.json
Interleaves variants in rounds inside one process (cdna_hip_programming.md
5.4 rule 24) and reports the median and min per variant.
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "membench.json"
    L = _lib.load()
    D = _lib.diag()
    eng = _lib.Engine(0)
    res = {"membench": {}, "hll_variants": {}}

    def mb(mode, buf, nbytes, nops):
        ms = ctypes.c_double()
        _lib.check_diag(D.rsk_diag_membench(eng.ctx, mode, buf.ptr, nbytes, nops, ctypes.byref(ms)))
        return ms.value

    rounds = 5
    big = devmem.DeviceBuffer(eng, 16 << 30)
    big.zero()
    cases = [
        ("stream_read_16GiB", 0, 16 << 30, 0, lambda ms: (16 << 30) / ms / 1e6, "GB/s"),
        ("stream_copy_8GiB_each_way", 3, 16 << 30, 0, lambda ms: (16 << 30) / ms / 1e6, "GB/s (read+write)"),
        ("stream_copy_split_8GiB_each_way", 7, 16 << 30, 0, lambda ms: (16 << 30) / ms / 1e6, "GB/s (read+write)"),
        ("stream_write_16GiB", 4, 16 << 30, 0, lambda ms: (16 << 30) / ms / 1e6, "GB/s"),
        ("stream_write_nt_16GiB", 5, 16 << 30, 0, lambda ms: (16 << 30) / ms / 1e6, "GB/s"),
        ("gather4B_1.2GB", 1, 1_198_132_298, 1 << 30, lambda ms: (1 << 30) / ms * 1e3, "gathers/s"),
        ("gather4B_128MB", 1, 128 << 20, 1 << 30, lambda ms: (1 << 30) / ms * 1e3, "gathers/s"),
        ("gather4B_2MB", 1, 2 << 20, 1 << 30, lambda ms: (1 << 30) / ms * 1e3, "gathers/s"),
        ("atomicor4B_1.2GB", 2, 1_198_132_298, 1 << 30, lambda ms: (1 << 30) / ms * 1e3, "atomics/s"),
        ("atomicor4B_128MB", 2, 128 << 20, 1 << 30, lambda ms: (1 << 30) / ms * 1e3, "atomics/s"),
        ("atomicor4B_2MB", 2, 2 << 20, 1 << 30, lambda ms: (1 << 30) / ms * 1e3, "atomics/s"),
    ]
    if os.environ.get("MEMBENCH_SKIP_MEM"):
        cases = []
    samples = {c[0]: [] for c in cases}
    for _ in range(rounds):
        for name, mode, nbytes, nops, rate, unit in cases:
            samples[name].append(rate(mb(mode, big, nbytes, nops)))
    for name, mode, nbytes, nops, rate, unit in cases:
        s = samples[name]
        res["membench"][name] = {"median": statistics.median(s), "max": max(s), "unit": unit}
        print(name, "%.4g %s (max %.4g)" % (statistics.median(s), unit, max(s)), flush=True)
    big.free()

    n = 1_000_000_000
    keys = devmem.gen_keys16(eng, 0x5EED0002, 0, n)
    names = {0: "U4_T512_nt", 1: "U8_T512_nt", 2: "U2_T512_nt", 3: "U4_T512_plain", 4: "U4_T1024_nt",
             5: "U4_T256_nt", 6: "U8_T1024_nt", 7: "U2_T1024_nt", 8: "b8_U4_T512_4wg", 9: "b8_U4_T256_8wg",
             10: "b8_U8_T512_4wg", 11: "b8_U4_T1024_2wg", 12: "pf_U4_T256", 13: "pf_U2_T256", 14: "pf_U8_T256"}
    if os.environ.get("MEMBENCH_VARIANTS"):  # e.g. "5,12,13,14"
        keep = {int(x) for x in os.environ["MEMBENCH_VARIANTS"].split(",")}
        names = {v: nm for v, nm in names.items() if v in keep}
    vs = {v: [] for v in names}
    for _ in range(rounds):
        for v in names:
            ms = ctypes.c_double()
            _lib.check_diag(D.rsk_diag_hll_variant(eng.ctx, v, keys.ptr, n, ctypes.byref(ms)))
            vs[v].append(ms.value)
    for v, nm in names.items():
        med = statistics.median(vs[v])
        res["hll_variants"][nm] = {"median_ms": med, "min_ms": min(vs[v]), "GBps_median": 16 * n / med / 1e6}
        print(nm, "median %.3f ms  %.0f GB/s" % (med, 16 * n / med / 1e6), flush=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
