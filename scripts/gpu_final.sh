#!/bin/bash
# Round-end GPU session on the final tree: parity tests, smoke, the three
# bench workloads, rocprofv3 kernel stats of the headline bench, separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) for C2/C3 and for C5.  Each GPU step has its
# own limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step pytest_gpu 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_full 300 python bench.py || exit 1
step bench_c4 200 python bench.py --workload c4 || exit 1
step bench_c5 200 python bench.py --workload c5 || exit 1
rm -rf gpurun_out/prof_stats gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc5_fetch gpurun_out/pmc5_write
step prof_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu || exit 1
step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --bloom-keys 200000000 || exit 1
step pmc_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --bloom-keys 200000000 || exit 1
step pmc5_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc5_fetch -o run -- python3 bench.py --workload c5 --steps 2 --warmup 1 || exit 1
step pmc5_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc5_write -o run -- python3 bench.py --workload c5 --steps 2 --warmup 1 || exit 1
python scripts/pmc_summary.py gpurun_out/prof_stats gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/${TAG}_pmc 1000000000
python scripts/pmc_summary.py gpurun_out/prof_stats gpurun_out/pmc5_fetch gpurun_out/pmc5_write gpurun_out/${TAG}_pmc_c5 500000000
find gpurun_out/prof_stats -name "*stats.csv" -exec cp {} gpurun_out/ \;
exit 0
