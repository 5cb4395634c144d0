#!/bin/bash
# Round-6 GPU sessions (conventions of scripts/gpu_r03.sh: every GPU step under
# its own time limit, the first failure ends the script, no retries).
#   scripts/gpu_r05.sh PART[,PART...] [args]
#     tests   : the -m gpu suite (or the given test paths), then smoke
#     sel     : only the given test paths / -k expression
#     bench   : the default bench line (C2 + Bloom + C4/C5/C5-Zipf extras + CPU baselines)
#     benchq  : the same without the CPU baselines
#     c4|c5|c5z : one workload alone
#     calib   : FETCH_SIZE calibration per read pattern -> gpurun_out/r05_fetch_calib.json
#     prof    : kernel trace of the headline bench + its FETCH/WRITE passes (r05_pmc*)
#     prof4|prof5|prof5z : kernel trace + FETCH/WRITE passes of the C4 / C5 / C5-Zipf bench
#     replies : add() with replies alone under rocprofv3 (trace, FETCH, WRITE)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PART=${1:-tests}
shift || true
TAG=${TAG:-r06}
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
# kernel trace + FETCH + WRITE passes of one command, summarised by pmc_summary.py
profw() {  # name limit keys config_json cmd...
  local name=$1 lim=$2 keys=$3 cfg=$4; shift 4
  rm -rf gpurun_out/${name}_stats gpurun_out/${name}_fetch gpurun_out/${name}_write
  step ${name}_stats $lim rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${name}_stats -o run -- "$@" || return 1
  step ${name}_fetch $lim rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${name}_fetch -o run -- "$@" || return 1
  step ${name}_write $lim rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${name}_write -o run -- "$@" || return 1
  python3 scripts/pmc_summary.py gpurun_out/${name}_stats gpurun_out/${name}_fetch gpurun_out/${name}_write \
    gpurun_out/${TAG}_${name} "$keys" "$cfg" > /dev/null || return 1
  find gpurun_out/${name}_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_${name}_kernel_stats.csv \;
}
for p in ${PART//,/ }; do
  case $p in
    tests)
      step pytest_gpu 900 $PYT -m gpu ${@:-tests} || exit 1
      step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    sel)
      step pytest_sel 600 $PYT -m gpu "$@" || exit 1 ;;
    bench)
      step bench 500 python bench.py || exit 1 ;;
    benchq)
      step benchq 400 python bench.py --no-cpu || exit 1 ;;
    c4)
      step bench_c4 200 python bench.py --workload c4 || exit 1 ;;
    c5)
      step bench_c5 200 python bench.py --workload c5 || exit 1 ;;
    c5z)
      step bench_c5_zipf 200 python bench.py --workload c5 --zipf 1.1 || exit 1 ;;
    calib)
      rm -rf gpurun_out/calib_fetch
      step calib 120 python3 scripts/fetch_calib.py || exit 1
      step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o run -- python3 scripts/fetch_calib.py || exit 1
      python3 scripts/calib_summary.py gpurun_out/calib_fetch gpurun_out/${TAG}_fetch_calib.json > /dev/null || exit 1 ;;
    prof)
      profw pmc 300 1000000000 '{"workload": "c2", "keys": 1000000000, "zipf": 0.0, "bloom_keys": 1000000000}' \
        python3 bench.py --no-cpu --no-bloom-replies --no-extra || exit 1
      python3 scripts/prof_agree.py gpurun_out/pmc_stats gpurun_out/pmc_stats.log gpurun_out/${TAG}_roofline_check.json || true ;;
    prof4)
      profw pmc_c4 200 1000000000 '{"workload": "c4", "keys": 1000000000, "zipf": 0.0, "bloom_keys": 0}' \
        python3 bench.py --workload c4 --steps 10 --warmup 3 || exit 1 ;;
    prof5)
      profw pmc_c5 200 500000000 '{"workload": "c5", "keys": 500000000, "zipf": 0.0, "bloom_keys": 0}' \
        python3 bench.py --workload c5 --steps 10 --warmup 3 || exit 1 ;;
    prof5z)
      profw pmc_c5_zipf 200 500000000 '{"workload": "c5", "keys": 500000000, "zipf": 1.1, "bloom_keys": 0}' \
        python3 bench.py --workload c5 --zipf 1.1 --steps 10 --warmup 3 || exit 1 ;;
    gab)  # C5 grouped add, routes A/B interleaved: GAB="route=v,...;route=v,..." (uniform and Zipf 1.1)
      IFS=';' read -ra FORMS <<< "${GAB:-gpart_xcd=0;gpart_xcd=1}"
      for z in 0 1.1; do for rep in 1 2; do for f in "${FORMS[@]}"; do
        step gab_$rep 120 python3 scripts/gpart_profile.py 5 $z "$f" || exit 1
        grep '^{' gpurun_out/gab_$rep.log >> gpurun_out/gab.jsonl
      done; done; done ;;
    gtrace)  # kernel trace of the C5 grouped add alone (uniform and Zipf 1.1)
      for z in 0 1.1; do
        rm -rf gpurun_out/gtrace_$z
        step gtrace_$z 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gtrace_$z -o run -- python3 scripts/gpart_profile.py 5 $z || exit 1
      done ;;
    c4var)  # C4 kernel variants interleaved (VARIANTS=..., scripts/var_variants.py)
      step c4var 300 python3 scripts/var_variants.py gpurun_out/c4var.json || exit 1 ;;
    io)  # batched Redis export / import of the C5 pool alone
      step io 200 python3 scripts/io_profile.py 3 ${IO_MERGES:-0} || exit 1
      grep '^{' gpurun_out/io.log >> gpurun_out/${TAG}_io_profile.jsonl ;;
    ioab)  # export / import routes A/B interleaved, one process each: IOAB="route=v,...;route=v,..."
      IFS=';' read -ra FORMS <<< "${IOAB:-io_drain=0;io_drain=1}"
      for m in ${IO_MERGES:-0 100000}; do for rep in 1 2; do for f in "${FORMS[@]}"; do
        step ioab_$rep 200 python3 scripts/io_profile.py ${IO_REPS:-3} $m "$f" || exit 1
        grep '^{' gpurun_out/ioab_$rep.log >> gpurun_out/${TAG}_ioab.jsonl
      done; done; done ;;
    chain)  # the C3 per-key arithmetic alone, in registers, at C3's size and boundary sizes
      for d in 9585058378 2147483648 2147483649 4294967297 8589934592 8589934593 17179869189 1099511627773 9007199254740993 4611686018427387909; do
        step chain_$d 60 scripts/bloom_chain_bench $d 7 || exit 1
        grep '^{' gpurun_out/chain_$d.log >> gpurun_out/${TAG}_bloom_chain.jsonl
      done ;;
    insroutes)  # the C3 insert under diag routes, interleaved (INS="spec spec ...")
      step insroutes 300 python3 scripts/insert_routes.py gpurun_out/${TAG}_insert_routes.json ${INS:-default sa_hash=1 sa_hash=2} || exit 1 ;;
    sqacct)  # SQ / LDS counters (3 passes) of the C3 insert, the insert without hashes, add() with replies
      export ROUNDS=1
      PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
      PB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_ADDR_CONFLICT"
      PC="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_ATOMIC_RETURN SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM"
      for run in ${SQRUNS:-ins ins_h1 rp}; do
        case $run in
          ins) R="python3 scripts/insert_routes.py gpurun_out/sq_ins.json default" ;;
          ins_h1) R="python3 scripts/insert_routes.py gpurun_out/sq_ins_h1.json sa_hash=1" ;;
          rp) R="python3 scripts/reply_profile.py 1000000000 1" ;;
        esac
        for pass in a b c; do
          case $pass in a) C=$PA ;; b) C=$PB ;; c) C=$PC ;; esac
          rm -rf gpurun_out/sq_${run}_$pass
          step sq_${run}_$pass 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sq_${run}_$pass -o run -- $R || exit 1
        done
      done ;;
    rpab)  # add() with replies, routes A/B interleaved, one process each: RPAB="route=v,...;route=v,..."
      IFS=';' read -ra FORMS <<< "${RPAB:-reply_dbg=0;reply_dbg=4}"
      for rep in 1 2 3; do for f in "${FORMS[@]}"; do
        step rpab_$rep 120 python3 scripts/reply_profile.py 1000000000 2 "$f" || exit 1
        grep '^{' gpurun_out/rpab_$rep.log >> gpurun_out/${TAG}_rpab.jsonl
      done; done ;;
    chain1)
      step chain1 60 scripts/bloom_chain_bench || exit 1
      grep '^{' gpurun_out/chain1.log >> gpurun_out/${TAG}_bloom_chain.jsonl ;;
    c5tl)  # C5 bench step timeline: kernel + memory-copy trace
      rm -rf gpurun_out/c5tl
      step c5tl 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/c5tl -o run -- python3 bench.py --workload c5 --steps 5 --warmup 2 || exit 1 ;;
    replies)
      profw pmc_replies 200 1000000000 '{"workload": "bloom_add_replies", "keys": 1000000000, "zipf": 0.0, "bloom_keys": 1000000000}' \
        python3 scripts/reply_profile.py 1000000000 1 || exit 1 ;;
    routed)  # the routed add at C5 size through the self exchange, heavy pre-combine on / off, uniform and Zipf
      for z in 0 1.1; do for rep in 1 2; do for f in "" "route_heavy=-1"; do
        step routed_$rep 150 python3 scripts/routed_profile.py 3 $z "$f" || exit 1
        grep '^{' gpurun_out/routed_$rep.log >> gpurun_out/${TAG}_routed.jsonl
      done; done; done ;;
    d2hx)  # the link / host-copy probe in two successive processes, then the export twice (process-order effects)
      for rep in 1 2; do
        step d2h_$rep 120 python3 scripts/d2h_probe.py || exit 1
        grep '^{' gpurun_out/d2h_$rep.log >> gpurun_out/${TAG}_d2h_probe.jsonl
      done ;;
    p2p)  # >2 GB self send/recv probe (rsk_diag_p2p_probe): one uint8 / one uint64 transfer / 1 GiB pieces
      step p2p 300 python3 scripts/p2p_probe.py $P2P_SIZES || exit 1
      grep '^{' gpurun_out/p2p.log >> gpurun_out/${TAG}_p2p_probe.jsonl ;;
    *) echo "unknown part $p"; exit 2 ;;
  esac
done
exit 0
