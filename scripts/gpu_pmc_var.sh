#!/bin/bash
# PMC passes over the C4 PFADD kernel variants (scripts/var_variants.py, 200M keys).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 scripts/var_variants.py gpurun_out/vv.json 200000000"
rm -rf gpurun_out/pv_a gpurun_out/pv_b gpurun_out/pv_c
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pv_a -o run -- $T > gpurun_out/pv_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pv_b -o run -- $T > gpurun_out/pv_b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pv_c -o run -- $T > gpurun_out/pv_c.log 2>&1 || exit 1
python3 scripts/pmc_table.py gpurun_out/pv_a gpurun_out/pv_b gpurun_out/pv_c --kernels=var
