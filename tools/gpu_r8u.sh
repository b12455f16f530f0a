#!/bin/bash
# bundling-stream priority at N = 1: the 5 000-frame bench and config 4's 20 000-frame stream (K = 2 000,
# where the global solve's persistent grid needs nearly every CU slot)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
bash tools/gpu_envab.sh $T "BF_BA_HIGH_PRIORITY=0;--frames 20000" "BF_BA_HIGH_PRIORITY=1;--frames 20000" "BF_BA_HIGH_PRIORITY=0;" "BF_BA_HIGH_PRIORITY=1;"
