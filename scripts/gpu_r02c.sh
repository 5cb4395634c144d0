#!/bin/bash
# Super-tile knob sweep at 1B keys + PMC passes over the chosen config (same key count).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -6 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
step st_sweep 600 python3 scripts/bloom_part_tune.py gpurun_out/st_sweep.json 1000000000 "RSK_BLOOM_ST_T1=1024" "RSK_BLOOM_ST_T1=1024,RSK_BLOOM_ST_T2=512" "RSK_BLOOM_ST_T1=1024,RSK_BLOOM_ST_UA=8" "RSK_BLOOM_ST_T1=512,RSK_BLOOM_ST_T2=512,RSK_BLOOM_ST_UA=8" || exit 1
export RSK_BLOOM_ST_T1=1024
T="python3 scripts/bloom_part_tune.py gpurun_out/t.json 1000000000"
rm -rf gpurun_out/stp_*
step stp_a 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/stp_a -o run -- $T || exit 1
step stp_b 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/stp_b -o run -- $T || exit 1
step stp_c 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/stp_c -o run -- $T || exit 1
step stp_d 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/stp_d -o run -- $T || exit 1
step stp_k 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stp_k -o run -- $T || exit 1
python3 scripts/pmc_table.py gpurun_out/stp_a gpurun_out/stp_b gpurun_out/stp_c gpurun_out/stp_d --kernels=st > gpurun_out/st_pmc_table.txt
exit 0
