#!/bin/bash
# GPU-box check: parity tests, then smoke.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocminfo 2>/dev/null | grep -m3 -E "gfx950|Marketing Name" ; nproc) > gpurun_out/devinfo.txt || true
timeout -k 10 900 python -m pytest tests -m gpu -q -ra > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
cat gpurun_out/smoke.log | tail -5
exit $rc
