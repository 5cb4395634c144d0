#!/bin/bash
# Fused grouped PFCOUNT + Bloom append pipeline: HLL + Bloom GPU tests, C5 benches, Bloom A/B timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -4 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
step pytest_hb 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hll.py tests/test_gpu_bloom.py tests/test_gpu_comm.py || exit 1
step bench_c5 300 python bench.py --workload c5 --steps 5 --warmup 2 || exit 1
step bench_c5_zipf 300 python bench.py --workload c5 --zipf 1.1 --steps 5 --warmup 2 || exit 1
step sa_ab 600 python3 scripts/bloom_part_tune.py gpurun_out/sa_ab.json 1000000000 "" "RSK_BLOOM_SA=0" "" || exit 1
exit 0
