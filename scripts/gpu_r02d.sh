#!/bin/bash
# st2 timing experiments (RSK_BLOOM_ST2_DBG: results wrong by design) at 1B keys.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -8 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
step st2_dbg 600 python3 scripts/bloom_part_tune.py gpurun_out/st2_dbg.json 1000000000 "RSK_BLOOM_ST_T1=1024" "RSK_BLOOM_ST_T1=1024,RSK_BLOOM_ST2_DBG=5" "RSK_BLOOM_ST_T1=1024,RSK_BLOOM_ST2_DBG=4" "RSK_BLOOM_ST_T1=1024,RSK_BLOOM_ST2_DBG=2" "RSK_BLOOM_ST_T1=1024,RSK_BLOOM_ST2_DBG=1" "RSK_BLOOM_ST_T1=1024,RSK_BLOOM_ST2_DBG=3" "RSK_BLOOM_ST_T1=1024,RSK_BLOOM_ST_T2=512,RSK_BLOOM_ST2_DBG=5" || exit 1
exit 0
