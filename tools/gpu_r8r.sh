#!/bin/bash
# host pool: loop / queue / app GPU tests, bench lines (N = 1, G = 8, G = 8 async 2) and the host profile build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_recon_gpu.py tests/test_long_queue_gpu.py tests/test_app_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
bash tools/gpu_lag.sh $T "" "--rehearse-shards 8" "--rehearse-shards 8 --async-bundling 2" || exit 1
bash tools/gpu_envab.sh $T "BF_HIP_LIB=bundlefusion_amd/libbf_hip_hostprof.so;--rehearse-shards 8" "BF_HIP_LIB=bundlefusion_amd/libbf_hip_hostprof.so;" || exit 1
grep -h "host us per frame" gpurun_out/$T/e*.err
