#!/bin/bash
# New round-2 tests (Zipf C5 variant, estimator branches, RBatch bitset, JNI shim caller, full-size C5 batches) + C5 Zipf bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -4 "gpurun_out/$name.log" | cut -c1-3000; return $rc; }
step pytest_new 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_jni_shim.py tests/test_gpu_reference_junit.py "tests/test_gpu_hll.py::test_count_estimator_branches" "tests/test_gpu_hll.py::test_zipf_stream_matches_oracle_and_partitioned_add" "tests/test_gpu_hll.py::test_c5_zipf_full_size_hot_groups_bit_exact" "tests/test_gpu_hll.py::test_c5_full_size_group_sample_bit_exact" || exit 1
step bench_c5 300 python bench.py --workload c5 --steps 5 --warmup 1 || exit 1
step bench_c5_zipf 300 python bench.py --workload c5 --zipf 1.1 --steps 5 --warmup 1 || exit 1
exit 0
