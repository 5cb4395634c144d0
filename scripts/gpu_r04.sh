#!/bin/bash
# Round-4 GPU sessions (same conventions as scripts/gpu_r03.sh: each GPU step
# under its own time limit, the first failure ends the script, no retries).
#   scripts/gpu_r04.sh c4pmc   SQ counters of the C4 kernel variants (two PMC passes)
#                      rpprof  add() with replies under rocprofv3 (trace, FETCH, WRITE)
#                      gcal    FETCH_SIZE per random gather (calibration)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PART=${1:-c4pmc}
shift || true
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
for p in ${PART//,/ }; do
  case $p in
    c4pmc)
      export VARIANTS=${VARIANTS:-0,4} ROUNDS=1
      V="python3 scripts/var_variants.py gpurun_out/c4pmc_var.json"
      rm -rf gpurun_out/c4pmc_a gpurun_out/c4pmc_b
      step c4pmc_a 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL --output-format csv -d gpurun_out/c4pmc_a -o run -- $V || exit 1
      step c4pmc_b 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/c4pmc_b -o run -- $V || exit 1
      unset VARIANTS ROUNDS ;;
    rpprof)  # add() with replies alone: kernel trace, then FETCH_SIZE and WRITE_SIZE passes (profiles/r04_pmc_replies.*)
      R="python3 scripts/reply_profile.py 1000000000 1"
      rm -rf gpurun_out/rp_stats gpurun_out/rp_fetch gpurun_out/rp_write
      step rp_stats 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_stats -o run -- $R || exit 1
      step rp_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/rp_fetch -o run -- $R || exit 1
      step rp_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/rp_write -o run -- $R || exit 1 ;;
    rpsq)  # SQ counters of the reply pipeline's kernels (two PMC passes of 8 SQ counters)
      R="python3 scripts/reply_profile.py 1000000000 1"
      rm -rf gpurun_out/rpsq_a gpurun_out/rpsq_b
      step rpsq_a 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/rpsq_a -o run -- $R || exit 1
      step rpsq_b 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --output-format csv -d gpurun_out/rpsq_b -o run -- $R || exit 1 ;;
    gcal)  # FETCH_SIZE of random gathers of known count (membench modes 1: 4 B gathers)
      rm -rf gpurun_out/gcal_fetch
      step gcal 120 python3 scripts/fetch_calib.py gathers || exit 1
      step gcal_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/gcal_fetch -o run -- python3 scripts/fetch_calib.py gathers || exit 1 ;;
    *) echo "unknown part $p"; exit 2 ;;
  esac
done
exit 0
