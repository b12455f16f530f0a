#!/bin/bash
# development loop on the GPU box: parity tests, timing probe, kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-dev}
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python tools/time_tsdf.py > gpurun_out/${TAG}_time.log 2>&1 || { echo "timing failed"; cat gpurun_out/${TAG}_time.log; exit 1; }
cat gpurun_out/${TAG}_time.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python tools/time_tsdf.py > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_prof/run_kernel_stats.csv
