#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T='tests/test_gpu_bloom.py::test_slice_routed_add_parity'
for d in 0 1 2 3; do
  echo "== dbg=$d"
  RSK_BLOOM_SA_DBG=$d timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu "$T" -k "SA" > gpurun_out/dbg_$d.log 2>&1
  rc=$?; tail -2 gpurun_out/dbg_$d.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
