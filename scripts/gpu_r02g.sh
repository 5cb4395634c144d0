#!/bin/bash
# Round-2 check of the current tree: full GPU suite, then the default bench (C2 + C3 incl. replies + CPU baselines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-3000; return $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step bench_full 600 python bench.py || exit 1
exit 0
