#!/bin/bash
# One GPU-box session: parity tests, smoke, runtime probe, bench, rocprof stats.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocminfo 2>/dev/null | grep -m3 -E "gfx950|Marketing Name" ; nproc) > gpurun_out/devinfo.txt || true
step() { local name=$1 lim=$2; shift 2; echo "== $name" ; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -4 "gpurun_out/$name.log"; return $rc; }
step pytest_gpu 900 python -m pytest tests -m gpu -q -ra -x || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step probe 300 python scripts/runtime_probe.py || exit 1
step bench_small 600 python bench.py --keys 200000000 --bloom-keys 200000000 --cpu-sample 16777216 --cpu-passes 1 || exit 1
exit 0
