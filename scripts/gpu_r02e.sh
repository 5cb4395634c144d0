#!/bin/bash
# C4 analysis: multiply throughput microbenchmark, the C4 bench, PMC of hll_add_var at 1B keys.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-1200; return $rc; }
hipcc -O3 --offload-arch=gfx950 -o /tmp/mul_bench scripts/mul_bench.hip > gpurun_out/mul_build.log 2>&1 || exit 1
step mul_bench 120 /tmp/mul_bench || exit 1
step bench_c4 600 python bench.py --workload c4 --steps 5 --warmup 1 || exit 1
T="python3 bench.py --workload c4 --steps 2 --warmup 1"
rm -rf gpurun_out/c4p_*
step c4p_a 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/c4p_a -o run -- $T || exit 1
step c4p_d 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/c4p_d -o run -- $T || exit 1
python3 scripts/pmc_table.py gpurun_out/c4p_a gpurun_out/c4p_d --kernels=hll_add_var > gpurun_out/c4_pmc_table.txt
exit 0
