#!/bin/bash
# Round-2 end-of-round GPU session on the final tree: parity suite, smoke, the
# bench workloads, rocprofv3 kernel trace of the headline bench (agreement of
# the trace with the bench's own HIP-event roofline), and separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) at the bench's own configuration; the same for the
# Bloom add()-with-replies pipeline alone (PART=replies).  Each GPU step has
# its own limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
PART=${2:-all}
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
if [ "$PART" = all ] || [ "$PART" = tests ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit 1
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
  step bench_full 400 python bench.py || exit 1
  step bench_c4 200 python bench.py --workload c4 || exit 1
  step bench_c5 200 python bench.py --workload c5 || exit 1
  step bench_c5_zipf 200 python bench.py --workload c5 --zipf 1.1 || exit 1
fi
if [ "$PART" = all ] || [ "$PART" = prof ]; then
  B="python3 bench.py --no-cpu --no-bloom-replies"
  rm -rf gpurun_out/prof_stats gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc5_fetch gpurun_out/pmc5_write
  step prof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- $B || exit 1
  python3 scripts/prof_agree.py gpurun_out/prof_stats gpurun_out/prof_bench.log gpurun_out/${TAG}_roofline_check.json
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $B || exit 1
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $B || exit 1
  FETCH_CALIB='{"segment_256B": 2.0}' python3 scripts/pmc_summary.py gpurun_out/prof_stats gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/${TAG}_pmc 1000000000 \
    '{"workload": "c2", "keys": 1000000000, "zipf": 0.0, "bloom_keys": 1000000000}'
  C5="python3 bench.py --workload c5"
  step prof5 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5_stats -o run -- $C5 || exit 1
  step pmc5_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc5_fetch -o run -- $C5 || exit 1
  step pmc5_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc5_write -o run -- $C5 || exit 1
  python3 scripts/pmc_summary.py gpurun_out/prof5_stats gpurun_out/pmc5_fetch gpurun_out/pmc5_write gpurun_out/${TAG}_pmc_c5 500000000 \
    '{"workload": "c5", "keys": 500000000, "zipf": 0.0, "bloom_keys": 0}'
  find gpurun_out/prof_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
  find gpurun_out/prof5_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_c5_kernel_stats.csv \;
fi
if [ "$PART" = all ] || [ "$PART" = prof ] || [ "$PART" = replies ]; then
  # add() with replies alone in its process (its sa1/sa2 instances share the
  # insert's kernel names)
  R="python3 scripts/reply_profile.py 1000000000 2"
  rm -rf gpurun_out/profr_stats gpurun_out/pmcr_fetch gpurun_out/pmcr_write
  step reply_bench 200 $R || exit 1
  step profr 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profr_stats -o run -- $R || exit 1
  step pmcr_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcr_fetch -o run -- $R || exit 1
  step pmcr_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcr_write -o run -- $R || exit 1
  python3 scripts/pmc_summary.py gpurun_out/profr_stats gpurun_out/pmcr_fetch gpurun_out/pmcr_write gpurun_out/${TAG}_pmc_replies 1000000000 \
    '{"workload": "bloom_add_replies", "keys": 1000000000, "zipf": 0.0, "bloom_keys": 1000000000}'
  find gpurun_out/profr_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_replies_kernel_stats.csv \;
fi
exit 0
