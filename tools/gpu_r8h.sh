#!/bin/bash
# preprocessing / app / loop tests, the G = 8 diagnosis (tools/gpu_g8.sh), the PCG phase timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_preprocess_gpu.py tests/test_recon_gpu.py tests/test_app_gpu.py tests/test_app_shards_gpu.py -x -v --timeout 600 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
bash tools/gpu_g8.sh $T $T || exit 1
bash tools/gpu_pcgtime.sh $T
