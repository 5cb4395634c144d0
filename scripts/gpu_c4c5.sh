set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c4 --steps 5 --warmup 1 > gpurun_out/bench_c4.log 2>&1; rc=$?; tail -2 gpurun_out/bench_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c5 --keys 500000000 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?; tail -2 gpurun_out/bench_c5.log; exit $rc
