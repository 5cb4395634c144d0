"""Issue accounting of one kernel from three rocprofv3 --pmc passes of SQ
counters (scripts/gpu_r05.sh sqacct): per-SIMD VALU busy, per-CU LDS and
scalar issue, against the kernel's cycles.

usage: sq_acct.py OUT.json KERNEL UNITS UNIT_NAME RUN=DIR_PREFIX [RUN=DIR_PREFIX ...]
  DIR_PREFIX: gpurun_out/sq_ins -> gpurun_out/sq_ins_{a,b,c}/run_counter_collection.csv

Counters are summed over the kernel's dispatches and divided by their number
(per launch).  Conventions (MI355X_MICROARCH.md):
  * SQ_BUSY_CYCLES is summed over the 32 shader engines: kernel cycles = / 32;
  * SQ_INSTS_VALU counts wave-instructions; one wave64 VALU instruction
    occupies a 16-lane SIMD 4 cycles at full rate, so 4 x INSTS_VALU / 1024
    SIMDs is the VALU busy time per SIMD with every instruction at full rate
    (a lower bound); SQ_INSTS_VALU_INT64 instructions (64-bit adds, shifts,
    v_mad_u64_u32) are the ones that may issue slower;
  * SQ_LDS_* cycle counters are summed over the 256 CUs: / 256 per CU;
  * SQ_INSTS_SALU: one scalar unit per CU, one instruction per cycle at best.
"""
import csv
import json
import sys
from collections import defaultdict

SES, CUS, SIMDS = 32, 256, 1024


def load(prefix, kernel):
    sums, disp, dur = defaultdict(float), defaultdict(set), {}
    for p in "abc":
        for row in csv.DictReader(open("%s_%s/run_counter_collection.csv" % (prefix, p))):
            name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            name = name.split("(")[0].split("<")[0].replace("rsk::", "")
            if name != kernel:
                continue
            sums[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[p].add(row["Dispatch_Id"])
            if p == "a":
                dur[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
    nd = max(len(v) for v in disp.values())
    c = {k: v / nd for k, v in sorted(sums.items())}
    c["kernel_ms_under_pmc"] = sum(dur.values()) / len(dur)
    return c, nd


def main():
    out, kernel, units, unit_name = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    runs = dict(a.split("=", 1) for a in sys.argv[5:])
    res = {"kernel": kernel, "units_per_launch": units, "unit": unit_name, "runs": {}}
    for run, prefix in runs.items():
        c, nd = load(prefix, kernel)
        cyc = c["SQ_BUSY_CYCLES"] / SES
        per = units / 64.0  # wave-instructions per 64 units
        acct = {
            "kernel_cycles (SQ_BUSY_CYCLES / 32 SEs)": cyc,
            "clock_GHz (kernel cycles / kernel_ms_under_pmc)": cyc / c["kernel_ms_under_pmc"] / 1e6,
            "valu_insts_per_64_units": c["SQ_INSTS_VALU"] / per,
            "valu_int64_insts_per_64_units": c.get("SQ_INSTS_VALU_INT64", 0) / per,
            "salu_insts_per_64_units": c["SQ_INSTS_SALU"] / per,
            "lds_insts_per_64_units": c["SQ_INSTS_LDS"] / per,
            "valu_busy_frac_per_simd (4 cycles / instruction)": 4 * c["SQ_INSTS_VALU"] / SIMDS / cyc,
            "valu_busy_frac_per_simd (INT64 at 16 cycles)": (4 * c["SQ_INSTS_VALU"] + 12 * c.get("SQ_INSTS_VALU_INT64", 0))
            / SIMDS / cyc,
            "salu_issue_frac_per_cu": c["SQ_INSTS_SALU"] / CUS / cyc,
            "lds_idx_active_frac_per_cu": c["SQ_LDS_IDX_ACTIVE"] / CUS / cyc,
            "lds_bank_conflict_frac_per_cu": c["SQ_LDS_BANK_CONFLICT"] / CUS / cyc,
            "lds_addr_conflict_frac_per_cu": c.get("SQ_LDS_ADDR_CONFLICT", 0) / CUS / cyc,
            "lds_atomic_return_frac_per_cu": c.get("SQ_LDS_ATOMIC_RETURN", 0) / CUS / cyc,
            "vmem_wr_issue_frac_per_cu": c.get("SQ_INST_CYCLES_VMEM_WR", 0) / CUS / cyc,
            "vmem_rd_issue_frac_per_cu": c.get("SQ_INST_CYCLES_VMEM_RD", 0) / CUS / cyc,
            "wave_frac_waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES)": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
            "wave_frac_issue_wait (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
        }
        res["runs"][run] = {"source": prefix + "_{a,b,c}", "dispatches": nd, "counters": c, "accounting": acct}
        print(run, {k: round(v, 3) for k, v in acct.items() if "frac" in k or "per_64" in k or "GHz" in k})
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
