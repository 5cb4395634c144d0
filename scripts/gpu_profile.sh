#!/bin/bash
# Full-size bench + rocprofv3 kernel stats + separate PMC passes (FETCH_SIZE,
# WRITE_SIZE).  Each GPU step has its own limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
KEYS=1000000000
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log"; return $rc; }
step bench_full 900 python bench.py || exit 1
rm -rf gpurun_out/prof_stats gpurun_out/pmc_fetch gpurun_out/pmc_write
step prof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu || exit 1
step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --bloom-keys 200000000 || exit 1
step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --bloom-keys 200000000 || exit 1
python scripts/pmc_summary.py gpurun_out/prof_stats gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/${TAG}_pmc $KEYS
find gpurun_out/prof_stats -name "*stats.csv" -exec cp {} gpurun_out/ \;
exit 0
