"""C4 (blob+offsets) PFADD kernel variants on the C4 stream, interleaved
rounds in one process: 0 production (step-count sort, 1 key per lane),
1 sorted, 2 keys per lane, 2 round-1 form, 3 sorted, 4 keys per lane; diagnostics of
the production kernel: 4 without MurmurHash64A, 5 without the register update, 6 without either;
7 the round-3 production form (ceil(len/8) classes, branch on the last block); 8 the LDS-DMA ring
form (the production route for short keys, C4).  VARIANTS=0,7 picks some.   python scripts/var_variants.py OUT.json [n]"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redisson_amd import _lib, devmem  # noqa: E402

NAMES = {0: "production_form2", 1: "sorted_2_per_lane", 2: "round1_simple", 3: "sorted_4_per_lane",
         4: "diag_trivial_hash", 5: "diag_no_update", 6: "diag_trivial_hash_no_update", 7: "round3_form",
         8: "ring_lds_dma", 9: "diag_ring_trivial_hash", 10: "staged_form1_unaligned_lds",
         11: "form2_stage20k_4wg", 12: "diag_stage20k_4wg_trivial_hash", 13: "form2_stage20k_3wg"}
if os.environ.get("VARIANTS"):
    NAMES = {int(v): NAMES[int(v)] for v in os.environ["VARIANTS"].split(",")}


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "var_variants.json"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
    L = _lib.load()
    D = _lib.diag()
    eng = _lib.Engine(0)
    blob, offs, tot = devmem.gen_varlen(eng, 0x5EED0005, 0, n)
    t = {v: [] for v in NAMES}
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for v in NAMES:
            ms = ctypes.c_double()
            _lib.check_diag(D.rsk_diag_hll_var_variant(eng.ctx, v, blob.ptr, offs.ptr, n, ctypes.byref(ms)))
            t[v].append(ms.value)
    res = {"n": n, "bytes": tot + 8 * n, "variants": {}}
    for v, nm in NAMES.items():
        med = statistics.median(t[v])
        res["variants"][nm] = {"median_ms": med, "min_ms": min(t[v]), "GBps": (tot + 8 * n) / med / 1e6}
        print("%-16s %8.3f ms  %.0f GB/s" % (nm, med, (tot + 8 * n) / med / 1e6), flush=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
