#!/bin/bash
# Super-tile Bloom insert: parity first, then stage timings at 1B keys.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -6 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
step pytest_st 600 python -u -m pytest tests/test_gpu_bloom.py -x -q --timeout 300 --timeout-method thread -k "slice_routed or partitioned or golden or c3_stream" || exit 1
step st_tune 600 python3 scripts/bloom_part_tune.py gpurun_out/st_tune.json 1000000000 "" "RSK_BLOOM_PG_T1=1024" "RSK_BLOOM_PG_T2=512" || exit 1
exit 0
