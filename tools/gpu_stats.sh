#!/bin/bash
# Parity tests of the TSDF path, then the kernel-time profile of the default bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-stats}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_tsdf_gpu.py tests/test_recon_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/${TAG}/pytest.log | head -20; tail -30 gpurun_out/${TAG}/pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}/pytest.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/$TAG/stats_bench.json 2> gpurun_out/$TAG/stats_bench.err || { echo "stats pass failed"; tail -20 gpurun_out/$TAG/stats_bench.err; exit 1; }
python3 tools/prof_summary.py gpurun_out/$TAG/stats/run_kernel_stats.csv > gpurun_out/$TAG/kernel_stats.txt && head -22 gpurun_out/$TAG/kernel_stats.txt
rm -f gpurun_out/$TAG/stats/run_kernel_trace.csv
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}/stats_bench.json')); print('fps %.1f' % d['value'], 'apply_us %.1f' % d['roofline']['avg_launch_us'])"
