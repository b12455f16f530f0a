#!/bin/bash
# queue host-time change: loop / queue GPU tests, then bench lines (N = 1, G = 8 rehearsal)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_recon_gpu.py tests/test_long_queue_gpu.py tests/test_recon_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
bash tools/gpu_lag.sh $T "" "--rehearse-shards 8" "--rehearse-shards 8 --no-preprocess" "--rehearse-shards 8 --async-bundling 2"
