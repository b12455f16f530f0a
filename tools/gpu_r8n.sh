#!/bin/bash
# cache intensity at 8x8 tiles (tests + standalone times), then the PMC profile of the driver's
# workload (--steps 20 --warmup 5) for the bench line's traffic / VALU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_preprocess_gpu.py tests/test_cache.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/pre -o pre --output-format csv -- python3 tools/time_preproc.py 300 > gpurun_out/$T/pre.log 2>&1 || { echo "time_preproc failed"; tail -20 gpurun_out/$T/pre.log; exit 1; }
grep "us/frame" gpurun_out/$T/pre.log
python3 tools/prof_summary.py gpurun_out/$T/pre/pre_kernel_stats.csv > gpurun_out/$T/pre_kernels.txt; cat gpurun_out/$T/pre_kernels.txt
find gpurun_out/$T/pre -name "*trace.csv" -delete
bash tools/profile_bench.sh $T/prof --steps 20 --warmup 5 || exit 1
cat gpurun_out/$T/prof/traffic.json
