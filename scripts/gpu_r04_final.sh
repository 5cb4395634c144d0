#!/bin/bash
# Round-4 measurement session on the current tree (as scripts/gpu_r03_final.sh):
# the -m gpu suite and smoke, the bench workloads, then the profiles (kernel
# traces + separate PMC passes of the bench configurations, tag r04).  Each
# GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PART=${1:-all}
if [ "$PART" = all ] || [ "$PART" = tests ]; then
  bash scripts/gpu_r03.sh tests || exit 1
fi
if [ "$PART" = all ] || [ "$PART" = bench ]; then
  bash scripts/gpu_r03.sh bench,c4,c5,c5z || exit 1
fi
if [ "$PART" = all ] || [ "$PART" = prof ]; then
  bash scripts/gpu_final_r02.sh r04 prof || exit 1
fi
exit 0
