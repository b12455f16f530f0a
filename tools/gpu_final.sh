#!/bin/bash
# Round-end evidence on the final code: kernel stats + PMC passes (FETCH, WRITE, VALU) of k_apply_ops
# for the driver's default bench command (--steps 50) and for --steps 20, then the -m gpu suite,
# smoke() and the default bench line (which takes traffic from the matching committed profile).
# Usage: tools/gpu_final.sh TAG [profiles|check|all]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-final}; WHAT=${2:-all}
if [ "$WHAT" != check ]; then
  bash tools/profile_bench.sh ${TAG}_s50 || exit 1
  bash tools/profile_bench.sh ${TAG}_s20 --steps 20 --warmup 5 || exit 1
fi
if [ "$WHAT" != profiles ]; then
  bash tools/gpu_check.sh ${TAG}_check || exit 1
fi
