#!/bin/bash
# Round-2 first GPU session: parity tests (new comm tests), the default bench,
# LDS-op throughput, and PMC passes over the C3 Bloom insert at 1B keys (the
# same key count as its stage timings).  Each GPU step has its own limit; the
# first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step bench_c2 600 python bench.py || exit 1
hipcc -O3 --offload-arch=gfx950 -o /tmp/lds_ops_bench scripts/lds_ops_bench.hip > gpurun_out/lds_build.log 2>&1 || exit 1
step lds_ops 120 /tmp/lds_ops_bench || exit 1
T="python3 scripts/bloom_part_tune.py gpurun_out/t.json 1000000000"
step bloom_tune 300 $T || exit 1
rm -rf gpurun_out/pmc_a gpurun_out/pmc_b gpurun_out/pmc_c gpurun_out/pmc_d
step pmc_a 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_a -o run -- $T || exit 1
step pmc_b 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_b -o run -- $T || exit 1
step pmc_c 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c -o run -- $T || exit 1
step pmc_d 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_d -o run -- $T || exit 1
python3 scripts/pmc_table.py gpurun_out/pmc_a gpurun_out/pmc_b gpurun_out/pmc_c gpurun_out/pmc_d --kernels=bloom > gpurun_out/bloom_pmc_table.txt
exit 0
