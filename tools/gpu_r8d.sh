#!/bin/bash
# new tests, the full GPU suite + smoke + default bench, then the loop trace and the k_apply_ops mask A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; SEL=$2
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest $SEL -x -v --timeout 300 --timeout-method thread > $O/first.log 2>&1 || { echo "first tests failed"; tail -40 $O/first.log; exit 1; }
tail -1 $O/first.log
bash tools/gpu_check.sh $TAG || exit 1
bash tools/gpu_r8c.sh $TAG
