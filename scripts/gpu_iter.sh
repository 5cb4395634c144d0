#!/bin/bash
# Iteration check: GPU parity tests, then the benches named in $@ (c2|c4|c5|variants|bloomvar).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for w in "$@"; do
  case $w in
    c2) timeout -k 10 600 python bench.py --no-cpu --no-bloom > gpurun_out/bench_c2.log 2>&1 ;;
    c4) timeout -k 10 600 python bench.py --workload c4 --steps 5 --warmup 1 > gpurun_out/bench_c4.log 2>&1 ;;
    c5) timeout -k 10 600 python bench.py --workload c5 --keys 500000000 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1 ;;
    variants) MEMBENCH_SKIP_MEM=1 timeout -k 10 600 python scripts/membench.py gpurun_out/variants.json > gpurun_out/bench_variants.log 2>&1 ;;
    bloomvar) timeout -k 10 600 python scripts/bloom_variants.py gpurun_out/bloom_variants.json > gpurun_out/bench_bloomvar.log 2>&1 ;;
  esac
  rc=$?; echo "== $w rc=$rc"; tail -14 gpurun_out/bench_$w.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
done
