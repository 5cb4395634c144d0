#!/bin/bash
# GPU session: parity tests, smoke, then the benches named in $@
# (c2 = full default bench line, c4, c5, c5prof, bloomvar).  Each GPU step has
# its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; tail -3 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for w in "$@"; do
  case $w in
    c2) step bench_c2 900 python bench.py || exit 1 ;;
    c4) step bench_c4 600 python bench.py --workload c4 --steps 5 --warmup 1 || exit 1 ;;
    c5) step bench_c5 600 python bench.py --workload c5 --keys 500000000 --steps 3 --warmup 1 || exit 1 ;;
    c5prof) step c5prof 600 python scripts/c5_profile.py || exit 1 ;;
    bloomvar) step bloomvar 600 python scripts/bloom_variants.py gpurun_out/bloom_variants.json || exit 1 ;;
    varvar) step varvar 600 python scripts/var_variants.py gpurun_out/var_variants.json || exit 1 ;;
  esac
done
exit 0
