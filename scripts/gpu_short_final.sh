#!/bin/bash
# Short round-end check on the final tree: parity tests, smoke, the headline
# bench and its rocprofv3 kernel stats.  Each GPU step has its own limit; the
# first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step pytest_gpu 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_full 300 python bench.py || exit 1
rm -rf gpurun_out/prof_stats
step prof_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu || exit 1
find gpurun_out/prof_stats -name "*stats.csv" -exec cp {} gpurun_out/ \;
exit 0
