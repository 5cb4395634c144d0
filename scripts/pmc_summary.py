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
hll_add16 kernel (the correction is recorded next to the raw value); every
other kernel takes the factor calibrated for its read pattern (READS below).
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


# Bytes per FETCH_SIZE byte by read pattern (MI355X_MICROARCH.md HBM: "calibrate
# on a known byte count in your own access pattern"), from scripts/fetch_calib.py
# under rocprofv3 (profiles/r05_fetch_calib.json; r03 for the uint4 patterns).
def load_calib():
    cal = {}
    for name in ("r03_fetch_calib.json", "r05_fetch_calib.json"):
        p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", name)
        if os.path.exists(p):
            for k, v in json.load(open(p)).get("patterns", {}).items():
                cal[k] = v["bytes_over_fetch_bytes"]
    # random 4-byte gathers: FETCH_SIZE counts 64 B per gather (profiles/r04_gather_fetch_calib.json,
    # 63.98 B raw per gather); the line fetched is taken as those 64 B (factor 1)
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                     "r04_gather_fetch_calib.json")
    if os.path.exists(p):
        cal["gather_64B"] = 1.0
    cal.update(json.loads(os.environ.get("FETCH_CALIB", "{}")))
    return cal


# Read pattern of each kernel's dominant loads: a pattern name, or a list of
# (pattern, share of the algorithmic read bytes) for kernels with two streams.
READS = {
    "hll_add16_kernel": "stream_read",                     # 16 B/lane nontemporal key stream
    "hll_add_var_staged_kernel": "stream_read",            # C4: 16 B/lane coalesced tile staging (blob + offsets)
    "hll_gpart1t_kernel": [("stream_read", 0.8), ("stream4_read", 0.2)],  # 16 B keys + 4 B group ids per pair
    "hll_gpart1_kernel": [("stream_read", 0.8), ("stream4_read", 0.2)],
    "hll_gcount_kernel": "stream_read",                    # uint4 id loads
    "hll_gcount2t_kernel": "segment4_128B",                # ~33-record segments, one dword per lane
    "hll_gpart2t_kernel": "segment4_128B",
    "hll_gcount2p_kernel": "stream_read",                  # uint4 run loads
    "hll_gpart2p_kernel": "stream_read",
    "hll_gapply_kernel": "stream_read",                    # uint4 loads of each fine bin's contiguous run
    "hll_gapply_extra_kernel": "stream_read",              # uint4 loads of a hot bin's extra chunks (round 5)
    # the Bloom add() with replies (rsk_bloom_reply.hip): rp1 = bloom_sa1 (16 B/lane keys), rp2 =
    # bloom_sa2h (uint4 sub-region reads), rp_tapply (uint4 segment loads), rp_treply (16 B/lane
    # keys + ~1.34 random 2-byte gathers of T per key, 64 B of FETCH each: gather_64B, r04 calibration)
    "bloom_sa1_kernel": "stream_read",
    "bloom_sa2h_kernel": "stream_read",
    "rp_tapply_kernel": "segment_256B",
    "rp_treply_kernel": [("stream_read", 0.16), ("gather_64B", 0.84)],
}


def read_factor(kernel, cal):
    pat = READS.get(kernel)
    if pat is None:
        return 1.0, "raw (uncalibrated pattern)"
    if isinstance(pat, str):
        pat = [(pat, 1.0)]
    if not all(p in cal for p, _ in pat):
        return 1.0, "raw (no calibration for %s)" % ", ".join(p for p, _ in pat if p not in cal)
    # corrected = raw x (sum of shares) / (sum of share / factor): each stream's raw share scaled by its factor
    f = sum(w for _, w in pat) / sum(w / cal[p] for p, w in pat)
    return f, " + ".join("%s x%.3f (%.0f%%)" % (p, cal[p], 100 * w) for p, w in pat)


def main():
    sdir, fdir, wdir, prefix, keys = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5])
    config = json.loads(sys.argv[6]) if len(sys.argv) > 6 else None
    cal = load_calib()
    st, sp = stats(sdir)
    fe, fp = counters(fdir, "FETCH_SIZE")
    wr, wp = counters(wdir, "WRITE_SIZE")
    kern = {}
    for k in sorted(set(st) | set(fe) | set(wr)):
        e = dict(st.get(k, {}))
        if k in fe:
            e["FETCH_SIZE_kib_raw"] = fe[k]
            f, how = read_factor(k, cal)
            e["fetch_bytes_corrected"] = fe[k] * 1024 * f
            e["fetch_correction"] = how
        if k in wr:
            e["WRITE_SIZE_kib"] = wr[k]
        if k == "hll_add16_kernel":
            e["keys_per_launch"] = keys
            e["algorithmic_bytes_per_launch"] = 16 * keys
            if k in fe:
                e["fetch_bytes_per_launch"] = e["fetch_bytes_corrected"]  # gfx950 wide-stream correction
            if k in fe and k in wr:
                e["hbm_bytes_per_launch"] = e["fetch_bytes_per_launch"] + wr[k] * 1024
        if k == "hll_add_var_staged_kernel" and k in fe and k in wr:
            e["keys_per_launch"] = keys
            e["hbm_bytes_per_launch"] = e["fetch_bytes_corrected"] + wr[k] * 1024
            e["hbm_bytes_note"] = "FETCH_SIZE x %s + WRITE_SIZE" % e["fetch_correction"]
            kern["hll_add_var_kernel"] = e  # bench.py's label of the C4 launch
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
        # the partitioned grouped PFADD as one unit (only in a C5-only run): per
        # stage, FETCH corrected by its read pattern's calibration, plus WRITE
        raw = sum((fe[p] + wr[p]) * 1024 for p in parts)
        kern["hll_add_grouped_partitioned"] = {
            "keys_per_launch": keys, "algorithmic_bytes_per_launch": 20 * keys,
            "hbm_bytes_per_launch": sum(kern[p]["fetch_bytes_corrected"] + wr[p] * 1024 for p in parts),
            "hbm_bytes_raw": raw,
            "stages": {p: {"fetch_bytes_corrected": kern[p]["fetch_bytes_corrected"],
                           "write_bytes": wr[p] * 1024, "fetch_correction": kern[p]["fetch_correction"],
                           "avg_ns": kern[p].get("avg_ns")} for p in parts},
            "hbm_bytes_note": "per call: every stage's FETCH_SIZE corrected by the calibrated factor of its read "
                              "pattern (scripts/fetch_calib.py) + WRITE_SIZE (exact for 16 B stores; raw for the "
                              "fine-bin pass's 4 B scattered stores)"}
    # add() with replies as one unit (a reply_profile.py run: one call per dispatch of each stage)
    rp = ("bloom_sa1_kernel", "sah_size_kernel", "st_offsets_kernel", "bloom_sa2h_kernel", "rp_tapply_kernel",
          "rp_treply_kernel")
    if "rp_treply_kernel" in kern and all(x in fe and x in wr for x in rp if x.startswith(("bloom_", "rp_"))):
        kern["bloom_add_replies"] = {
            "keys_per_launch": keys,
            "hbm_bytes_per_launch": sum(kern[x].get("fetch_bytes_corrected", 0.0) + wr.get(x, 0.0) * 1024
                                        for x in rp if x in kern),
            "hbm_bytes_raw": sum((fe.get(x, 0.0) + wr.get(x, 0.0)) * 1024 for x in rp),
            "stages": {x: {"fetch_bytes_corrected": kern[x].get("fetch_bytes_corrected"),
                           "write_bytes": wr.get(x, 0.0) * 1024, "fetch_correction": kern[x].get("fetch_correction"),
                           "avg_ns": kern[x].get("avg_ns")} for x in rp if x in kern},
            "hbm_bytes_note": "per add() call: FETCH_SIZE of each stage corrected by its read pattern's calibration "
                              "(rp_treply: keys x2, T gathers at 64 B each) + WRITE_SIZE"}
    # The Bloom insert at 1B keys, k = 7 (one chunk: one dispatch of each stage per insert call),
    # per stage and summed.  Append pipeline (default): sa1 reads the keys, sa2 its sub-regions and
    # apply its tiles with 16 B/lane loads, so FETCH is doubled per the guide; the header pipeline
    # (st1/st2/st_apply, RSK_BLOOM_SA=0) reads probe tags with 4 B loads (uncalibrated: raw).
    # Round 3: sa2 writes 16-bit records (bloom_sa2h_kernel) that bloom_sah_apply_kernel reads with
    # quarter-wave 256 B segment loads; the doubling is applied to it only as far as
    # scripts/fetch_calib.py shows it holds for that pattern (FETCH_CALIB, below).
    calib = cal
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
           "calibration": cal,
           "note": "FETCH_SIZE/WRITE_SIZE in KiB per dispatch (mean over dispatches); fetch_bytes_corrected = "
                   "FETCH_SIZE x the calibrated factor of the kernel's read pattern (MI355X_MICROARCH.md HBM)"}
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
