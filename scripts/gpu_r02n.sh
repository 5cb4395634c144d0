#!/bin/bash
# Bloom append pipeline v2 (per-workgroup sub-regions): parity, then A/B timing and PMC of sa1 vs st1 at 1B keys.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -5 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
step pytest_bloom 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bloom.py -k "slice_routed or c3" || exit 1
step sa_ab 600 python3 scripts/bloom_part_tune.py gpurun_out/sa_ab.json 1000000000 "" "RSK_BLOOM_SA=0" "" || exit 1
exit 0
T="python3 scripts/bloom_part_tune.py gpurun_out/t.json 1000000000 RSK_BLOOM_SA=1 RSK_BLOOM_SA=0"
rm -rf gpurun_out/sap_*
step sap_a 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/sap_a -o run -- $T || exit 1
step sap_b 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sap_b -o run -- $T || exit 1
step sap_c 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/sap_c -o run -- $T || exit 1
step sap_d 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sap_d -o run -- $T || exit 1
python3 scripts/pmc_table.py gpurun_out/sap_a gpurun_out/sap_b gpurun_out/sap_c gpurun_out/sap_d --kernels=bloom_s > gpurun_out/sap_pmc_table.txt
exit 0
