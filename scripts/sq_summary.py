"""Per-kernel SQ counter summary of one rocprofv3 --pmc pass.

usage: sq_summary.py COUNTER_CSV OUT.json KEYS_PER_DISPATCH "SOURCE TEXT" [KERNEL_SUBSTR ...]

Sums every counter per kernel over its dispatches and divides by the number
of dispatches, so the figures are per launch; `*_insts_per_64_keys` divides
the instruction counts by KEYS_PER_DISPATCH / 64 (wave-instructions per 64
keys, i.e. per wave-worth of keys).  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_*
count quad-cycles on gfx950 (MI355X_MICROARCH.md), so only their ratios are
quoted.
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, out, keys, source = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    only = sys.argv[5:]
    sums = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0].split("<")[0].replace("rsk::", "")
        if only and not any(s in name for s in only):
            continue
        sums[name][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[name].add(row["Dispatch_Id"])
    res = {}
    for name, c in sums.items():
        nd = len(disp[name])
        k = {n: v / nd for n, v in sorted(c.items())}
        k["dispatches"] = nd
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM"):
            if n in k:
                k[n.replace("SQ_INSTS_", "").lower() + "_insts_per_64_keys"] = k[n] / (keys / 64)
        wc = k.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_ANY"):
                if n in k:
                    k["frac_" + n.replace("SQ_", "").lower()] = k[n] / wc
        res[name] = k
    json.dump({"source": source, "keys_per_dispatch": keys, "kernels": res}, open(out, "w"), indent=1)
    for name, k in sorted(res.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(name, {n: round(v, 3) for n, v in k.items() if n.startswith(("frac", "valu", "lds", "salu"))})


if __name__ == "__main__":
    main()
