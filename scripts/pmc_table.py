"""Per-kernel mean of every counter in one or more rocprofv3 --pmc output dirs.

    python scripts/pmc_table.py DIR [DIR ...] [--kernels substr,substr]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = []
    for a in sys.argv[1:]:
        if a.startswith("--kernels="):
            filt = a.split("=", 1)[1].split(",")
    vals = defaultdict(lambda: defaultdict(list))
    for d in args:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(p)):
                k = short(row["Kernel_Name"])
                if filt and not any(f in k for f in filt):
                    continue
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print("   %-28s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
