"""Check that the bench's roofline figure is reproducible from the profile.

usage: python scripts/prof_agree.py TRACE_DIR BENCH_LOG OUT.json [KERNEL]

TRACE_DIR: a `rocprofv3 --kernel-trace --stats --output-format csv` run of
the bench command; BENCH_LOG: that same process's stdout (its JSON line).
The last `steps` dispatches of KERNEL (default hll_add16_kernel) in the trace
are the bench's timed launches; their mean duration must agree with the
bench's own HIP-event mean (roofline.avg_launch_ms) from the same process.
Writes both, the rocprof stats average over all dispatches (warm-up
included), and the roofline fraction each implies."""
import csv
import glob
import json
import os
import sys


def main():
    tdir, blog, out = sys.argv[1], sys.argv[2], sys.argv[3]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "hll_add16_kernel"
    bench = json.loads([ln for ln in open(blog) if ln.startswith("{")][-1])
    trace = glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True)[0]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for r in csv.DictReader(open(trace)) if kernel in r["Kernel_Name"]]
    steps = bench["steps"]
    timed = durs[-steps:]
    rl = bench["roofline"]
    bytes_ = rl["algorithmic_bytes_per_launch"]
    trace_ms = sum(timed) / len(timed)
    res = {
        "kernel": kernel, "bench_steps": steps, "bench_warmup": bench["warmup"],
        "dispatches_in_trace": len(durs),
        "bench_hip_event_avg_ms": rl["avg_launch_ms"],
        "rocprof_trace_avg_ms_timed_dispatches": trace_ms,
        "rocprof_trace_all_dispatches_ms": durs,
        "rocprof_all_dispatch_avg_ms": sum(durs) / len(durs),
        "agreement": trace_ms / rl["avg_launch_ms"],
        "frac_bench": rl["frac"],
        "frac_from_trace": bytes_ / (trace_ms / 1e3) / 1e9 / rl["peak"],
        "algorithmic_bytes_per_launch": bytes_,
        "bench_ms_per_step": bench["ms_per_step"],
        "trace": os.path.relpath(trace),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "rocprof_trace_all_dispatches_ms"}))


if __name__ == "__main__":
    main()
