#!/bin/bash
# Heavy-bin split of the grouped apply: grouped tests, C5 uniform + Zipf benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -4 "gpurun_out/$name.log" | cut -c1-2500; return $rc; }
step pytest_grouped 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hll.py -k "grouped or zipf or c5" || exit 1
step bench_c5 300 python bench.py --workload c5 --steps 5 --warmup 1 || exit 1
step bench_c5_zipf 300 python bench.py --workload c5 --zipf 1.1 --steps 5 --warmup 1 || exit 1
exit 0
