#!/bin/bash
# ray-cast tests after the splat revert; G = 2 / 4 / 8 rehearsals; PMC profile of the default bench (--steps 50)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_raycast_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
bash tools/gpu_lag.sh $T "--rehearse-shards 8" "--rehearse-shards 4" "--rehearse-shards 2" "--rehearse-shards 8 --no-preprocess" || exit 1
bash tools/profile_bench.sh $T/s50 || exit 1
cat gpurun_out/$T/s50/traffic.json
