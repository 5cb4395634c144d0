"""FETCH_SIZE calibration summary: the dispatches of `scripts/fetch_calib.py`
under `rocprofv3 --pmc FETCH_SIZE` against the bytes each one read.

usage: python scripts/calib_summary.py FETCH_DIR OUT_JSON

Each fetch_calib case is one dispatch of a diag kernel over the same 4 GiB
buffer, every byte read exactly once; bytes_over_fetch_bytes is the factor
scripts/pmc_summary.py applies to a kernel whose loads follow that pattern.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fetch_calib import CASES  # noqa: E402

# the diag kernel (rsk_diag.hip) that serves each case, in the order fetch_calib.py runs them
KERNELS = {"stream_read": "diag_stream_read", "segment_256B": "diag_segment_read<16>",
           "segment_512B": "diag_segment_read<32>", "segment_1KiB": "diag_segment_read<64>",
           "stream4_read": "diag_read4<0>", "segment4_128B": "diag_read4<32>", "segment4_256B": "diag_read4<64>"}
NBYTES = 4 << 30


def main():
    fdir, out = sys.argv[1], sys.argv[2]
    p = glob.glob(os.path.join(fdir, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(p)) if r.get("Counter_Name") == "FETCH_SIZE"]
    pats = {}
    for name, _, _ in CASES:
        kn = KERNELS[name]
        hit = [float(r["Counter_Value"]) for r in rows if kn in r["Kernel_Name"].replace(" ", "")]
        if not hit:
            continue
        kib = hit[0]
        pats[name] = {"FETCH_SIZE_kib": kib, "bytes_over_fetch_bytes": NBYTES / (kib * 1024)}
    doc = {"bytes_read_per_dispatch": NBYTES,
           "source": "scripts/fetch_calib.py under rocprofv3 --pmc FETCH_SIZE (scripts/gpu_r05.sh calib)",
           "patterns": pats}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
