#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 120 python3 scripts/occ_probe.py && timeout -k 10 120 python3 scripts/occ_probe.py torch
