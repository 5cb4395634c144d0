#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step pytest_g 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hll.py -k "grouped or zipf or c5" || exit 1
step bench_c5_pc 300 python bench.py --workload c5 --steps 5 --warmup 2 || exit 1
RSK_HLL_PCOUNT=0 step bench_c5_nopc 300 python bench.py --workload c5 --steps 5 --warmup 2 || exit 1
step bench_c5_pc2 300 python bench.py --workload c5 --steps 5 --warmup 2 || exit 1
python3 - <<'PY'
import json
for f in ('bench_c5_pc','bench_c5_nopc','bench_c5_pc2'):
    d=json.loads([l for l in open('gpurun_out/%s.log'%f) if l.startswith('{')][-1])
    print(f, round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['roofline']['stage_ms_per_launch'].items()}, round(d['side_kernels_ms_per_launch']['hll_count'],3))
PY
exit 0
