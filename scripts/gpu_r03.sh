#!/bin/bash
# Round-3 GPU sessions.  Each GPU step runs under its own time limit and the
# first failure ends the script (no retries).
#   scripts/gpu_r03.sh PART [pytest selection...]
#     tests  : the -m gpu suite (or the given test paths), then smoke
#     sel    : only the given test paths / -k expression
#     bench  : bench.py (C2 headline + node Bloom + CPU baselines)
#     c4|c5|c5z : the other workloads
#     prof   : rocprofv3 kernel trace of the headline bench + PMC passes
#     insprof: the C3 insert under rocprofv3 (trace, FETCH, WRITE, SQ passes)
#     routes : scripts/insert_routes.py over the given route specs
#     calib  : FETCH_SIZE calibration per access pattern
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PART=${1:-tests}
shift || true
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for p in ${PART//,/ }; do
  case $p in
    tests)
      step pytest_gpu 900 $PYT -m gpu ${@:-tests} || exit 1
      step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    sel)
      step pytest_sel 600 $PYT -m gpu "$@" || exit 1 ;;
    bench)
      step bench 400 python bench.py || exit 1 ;;
    benchq)
      step benchq 300 python bench.py --no-cpu || exit 1 ;;
    c4)
      step bench_c4 200 python bench.py --workload c4 || exit 1 ;;
    c5)
      step bench_c5 200 python bench.py --workload c5 || exit 1 ;;
    c5z)
      step bench_c5_zipf 200 python bench.py --workload c5 --zipf 1.1 || exit 1 ;;
    routes)
      step routes 600 python -u scripts/insert_routes.py gpurun_out/ins_routes.json "$@" || exit 1 ;;
    replies)  # C3 add() with replies, 1B keys (scripts/reply_profile.py)
      step reply_bench 300 python3 scripts/reply_profile.py 1000000000 2 || exit 1 ;;
    c5prof)
      step c5prof 300 python scripts/c5_host_profile.py 500000000 1000000 10 || exit 1 ;;
    insprof)  # the reply-less C3 insert alone: kernel trace, then one PMC pass per counter group
      I="python3 scripts/insert_routes.py gpurun_out/ins_prof.json default"
      export ROUNDS=1
      rm -rf gpurun_out/ins_stats gpurun_out/ins_fetch gpurun_out/ins_write gpurun_out/ins_sq
      step ins_stats 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ins_stats -o run -- $I || exit 1
      step ins_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ins_fetch -o run -- $I || exit 1
      step ins_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ins_write -o run -- $I || exit 1
      step ins_sq 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/ins_sq -o run -- $I || exit 1
      unset ROUNDS ;;
    calib)  # FETCH_SIZE against known bytes per access pattern (scripts/fetch_calib.py)
      rm -rf gpurun_out/calib_fetch
      step calib 120 python3 scripts/fetch_calib.py || exit 1
      step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o run -- python3 scripts/fetch_calib.py || exit 1 ;;
    sq)  # SQ instruction / wait counters of the C5 and C4 kernels (one PMC pass each)
      SQC="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
      rm -rf gpurun_out/sq_c5 gpurun_out/sq_c4
      step sq_c5 200 rocprofv3 --pmc $SQC --output-format csv -d gpurun_out/sq_c5 -o run -- python3 bench.py --workload c5 --steps 3 --warmup 2 --no-cpu || exit 1
      step sq_c4 200 rocprofv3 --pmc $SQC --output-format csv -d gpurun_out/sq_c4 -o run -- python3 bench.py --workload c4 --steps 3 --warmup 2 --no-cpu || exit 1 ;;
    prof)
      B="python3 bench.py --no-cpu --no-bloom-replies"
      rm -rf gpurun_out/prof_stats
      step prof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- $B || exit 1 ;;
    *) echo "unknown part $p"; exit 2 ;;
  esac
done
exit 0
