#!/bin/bash
# Why is the Bloom insert slower inside bench.py than in the tuning script? A/B of the process context.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
step t_plain 300 python3 scripts/bloom_part_tune.py gpurun_out/t1.json 1000000000 "" || exit 1
RSK_TUNE_TORCH=1 step t_torch 300 python3 scripts/bloom_part_tune.py gpurun_out/t2.json 1000000000 "" || exit 1
RSK_TUNE_QBUF=1 step t_qbuf 300 python3 scripts/bloom_part_tune.py gpurun_out/t3.json 1000000000 "" || exit 1
step b_bloom 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-bloom-replies || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/b_bloom.log') if l.startswith('{')][-1]); print('bench', d['bloom']['insert_stage_ms'])"
exit 0
