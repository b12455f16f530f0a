#!/bin/bash
# The new/changed tests first (fail fast), then the full GPU check. Usage: tools/gpu_tests_first.sh TAG "pytest selectors" [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; SEL=$2; shift 2
mkdir -p gpurun_out/$TAG
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest $SEL -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/first.log 2>&1 || { echo "first tests failed"; tail -40 gpurun_out/$TAG/first.log; exit 1; }
  tail -1 gpurun_out/$TAG/first.log
fi
exec bash tools/gpu_check.sh $TAG "$@"
