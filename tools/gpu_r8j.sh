#!/bin/bash
# BA tests (the four-workgroup finisher), PCG phase timings, loop host time per frame
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest tests/test_ba_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
bash tools/gpu_pcgtime.sh $T || exit 1
bash tools/gpu_lag.sh $T "--rehearse-shards 8" "--rehearse-shards 8 --no-preprocess" "" "--rehearse-shards 8 --async-bundling 2"
