"""Summarise rocprofv3 output into profiles/*.json / *.md.

usage: python scripts/pmc_summary.py STATS_DIR FETCH_DIR WRITE_DIR OUT_PREFIX KEYS_PER_LAUNCH [CONFIG_JSON]

CONFIG_JSON ({"workload": "c2", "keys": 1e9, "bloom_keys": ..., "zipf": 0}) is
the bench configuration the three runs used; bench.py reads a summary's
traffic only when its own configuration equals it.

* STATS_DIR: rocprofv3 --kernel-trace --stats --output-format csv run
  (kernel_stats.csv: per-kernel calls / average duration).
* FETCH_DIR / WRITE_DIR: separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes
  (counter_collection.csv, one row per dispatch and counter).
HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane)
coalesced streaming read, so the read side is doubled for the streaming
hll_add16 kernel (the correction is recorded next to the raw value).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def find(d, pattern):
    hits = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return hits[0] if hits else None


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def stats(d):
    p = find(d, "*kernel_stats.csv")
    out = {}
    if not p:
        return out, None
    for row in csv.DictReader(open(p)):
        out[short(row["Name"])] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                   "total_ns": float(row["TotalDurationNs"]), "pct": float(row["Percentage"])}
    return out, p


def counters(d, counter):
    p = find(d, "*counter_collection.csv")
    vals = defaultdict(list)
    if not p:
        return {}, None
    for row in csv.DictReader(open(p)):
        if row.get("Counter_Name") != counter:
            continue
        vals[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, p


def main():
    sdir, fdir, wdir, prefix, keys = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5])
    config = json.loads(sys.argv[6]) if len(sys.argv) > 6 else None
    st, sp = stats(sdir)
    fe, fp = counters(fdir, "FETCH_SIZE")
    wr, wp = counters(wdir, "WRITE_SIZE")
    kern = {}
    for k in sorted(set(st) | set(fe) | set(wr)):
        e = dict(st.get(k, {}))
        if k in fe:
            e["FETCH_SIZE_kib_raw"] = fe[k]
        if k in wr:
            e["WRITE_SIZE_kib"] = wr[k]
        if k == "hll_add16_kernel":
            e["keys_per_launch"] = keys
            e["algorithmic_bytes_per_launch"] = 16 * keys
            if k in fe:
                e["fetch_bytes_per_launch"] = fe[k] * 1024 * 2  # gfx950 wide-stream correction
            if k in fe and k in wr:
                e["hbm_bytes_per_launch"] = e["fetch_bytes_per_launch"] + wr[k] * 1024
        if k == "hll_add_grouped16_kernel" and k in fe and k in wr:
            # mixed access (16 B key stream + 4 B group ids + random 4 B register
            # words): no calibrated correction exists, so the raw counters are used
            e["keys_per_launch"] = keys
            e["algorithmic_bytes_per_launch"] = 20 * keys
            e["hbm_bytes_per_launch"] = (fe[k] + wr[k]) * 1024
            e["hbm_bytes_note"] = "raw FETCH_SIZE + WRITE_SIZE (uncalibrated for random 4 B access)"
        kern[k] = e
    # tile-major form (default since late round 4) or the exact-offset form (route gpart_tm=0)
    parts = ("hll_gpart1t_kernel", "hll_hdr_transpose_kernel", "hll_gcount2t_kernel", "hll_gpart2t_kernel",
             "hll_gapply_kernel")
    if not all(p in fe and p in wr for p in parts):
        parts = ("hll_gcount_kernel", "hll_gpart1_kernel", "hll_gcount2p_kernel", "hll_gpart2p_kernel",
                 "hll_gapply_kernel")
    extras = tuple(p for p in ("hll_gextra_list_kernel", "hll_gapply_extra_kernel") if p in fe and p in wr)
    if "hll_gapply_kernel" in kern and all(p in fe and p in wr for p in parts):
        parts = parts + extras
        # the partitioned grouped PFADD as one unit (only in a C5-only run): raw
        # counters summed over its stages
        kern["hll_add_grouped_partitioned"] = {
            "keys_per_launch": keys, "algorithmic_bytes_per_launch": 20 * keys,
            "hbm_bytes_per_launch": sum((fe[p] + wr[p]) * 1024 for p in parts),
            "stages": list(parts),
            "hbm_bytes_note": "raw FETCH_SIZE + WRITE_SIZE of the stages per call (16 B key stream, 4 B records, "
                              "16 KiB sketch rows; not corrected)"}
    # The Bloom insert at 1B keys, k = 7 (one chunk: one dispatch of each stage per insert call),
    # per stage and summed.  Append pipeline (default): sa1 reads the keys, sa2 its sub-regions and
    # apply its tiles with 16 B/lane loads, so FETCH is doubled per the guide; the header pipeline
    # (st1/st2/st_apply, RSK_BLOOM_SA=0) reads probe tags with 4 B loads (uncalibrated: raw).
    # Round 3: sa2 writes 16-bit records (bloom_sa2h_kernel) that bloom_sah_apply_kernel reads with
    # quarter-wave 256 B segment loads; the doubling is applied to it only as far as
    # scripts/fetch_calib.py shows it holds for that pattern (FETCH_CALIB, below).
    calib = json.loads(os.environ.get("FETCH_CALIB", "{}"))
    for name, st, wide in (("bloom_insert_supertile",
                            ("bloom_sa1_kernel", "sah_size_kernel", "st_offsets_kernel", "bloom_sa2h_kernel",
                             "bloom_sah_apply_kernel"),
                            ("bloom_sa1_kernel", "bloom_sa2h_kernel") + (
                                ("bloom_sah_apply_kernel",) if calib.get("segment_256B", 1.0) > 1.5 else ())),
                           ("bloom_insert_header_pipeline",
                            ("bloom_st1_kernel", "st_transpose_kernel", "st_size_kernel", "st_offsets_kernel",
                             "bloom_st2_kernel", "bloom_st_apply_kernel"), ("bloom_st1_kernel",))):
        main = [x for x in st if x.startswith("bloom_")]
        if not all(x in fe and x in wr for x in main):
            continue
        stages = {x: {"fetch_kib_raw": fe.get(x, 0.0), "write_kib": wr.get(x, 0.0),
                      "avg_ns": kern.get(x, {}).get("avg_ns")} for x in st if x in fe}
        raw = sum((fe.get(x, 0.0) + wr.get(x, 0.0)) * 1024 for x in st)
        kern[name] = {"stages": stages, "hbm_bytes_per_insert_raw": raw,
                      "hbm_bytes_per_launch": raw + sum(fe[x] * 1024 for x in wide if x in fe),
                      "wide_read_stages_doubled": list(wide),
                      "note": "per insert call = one dispatch of each stage"}
    doc = {"config": config, "sources": {"stats": sp, "fetch": fp, "write": wp}, "kernels": kern,
           "note": "FETCH_SIZE/WRITE_SIZE in KiB per dispatch (mean over dispatches); fetch doubled for "
                   "hll_add16_kernel per MI355X_MICROARCH.md HBM section"}
    with open(prefix + ".json", "w") as f:
        json.dump(doc, f, indent=1)
    lines = ["| kernel | calls | avg us | % time | FETCH_SIZE KiB (raw) | WRITE_SIZE KiB |", "|---|---|---|---|---|---|"]
    for k, e in sorted(kern.items(), key=lambda kv: -kv[1].get("pct", 0)):
        lines.append("| %s | %s | %.1f | %.2f | %s | %s |" % (
            k, e.get("calls", ""), e.get("avg_ns", 0) / 1e3, e.get("pct", 0),
            "%.0f" % e["FETCH_SIZE_kib_raw"] if "FETCH_SIZE_kib_raw" in e else "",
            "%.0f" % e["WRITE_SIZE_kib"] if "WRITE_SIZE_kib" in e else ""))
    with open(prefix + ".md", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
