#!/bin/bash
# Bloom append pipeline (sa1/sa2): Bloom parity tests, then A/B timing at 1B keys (append vs header pipeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -6 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
step pytest_bloom 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bloom.py -k "slice_routed or c3" || exit 1
step sa_ab 600 python3 scripts/bloom_part_tune.py gpurun_out/sa_ab.json 1000000000 "" "RSK_BLOOM_SA_DBG=3" "RSK_BLOOM_SA=0" "RSK_BLOOM_ST_T1=1024" "" || exit 1
exit 0
