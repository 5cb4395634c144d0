#!/bin/bash
# C4 with LDS-only barriers: C4 tests, variants A/B, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -6 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
step pytest_c4 300 python -u -m pytest tests/test_gpu_hll.py tests/test_gpu_hll_staged.py -x -q --timeout 300 --timeout-method thread -k "var or varlen or c4 or fixed or staged" || exit 1
step varvar 600 python scripts/var_variants.py gpurun_out/var_variants.json || exit 1
step bench_c4 600 python bench.py --workload c4 --steps 10 --warmup 3 || exit 1
exit 0
