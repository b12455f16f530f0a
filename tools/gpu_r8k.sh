#!/bin/bash
# preprocessing / cache kernels (unrolled taps, interior fast path): parity tests, standalone kernel
# times; k_apply_ops grid with free workgroup slots for the bundling launches (A/B)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_preprocess_gpu.py tests/test_cache.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head; tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/pre -o pre -- python3 tools/time_preproc.py 300 > gpurun_out/$T/pre.log 2>&1 || { echo "time_preproc failed"; tail -20 gpurun_out/$T/pre.log; exit 1; }
grep "us/frame" gpurun_out/$T/pre.log
python3 tools/prof_summary.py $(find gpurun_out/$T/pre -name "*kernel_stats.csv" | head -1) 2>/dev/null | head -12
bash tools/gpu_envab.sh $T "BF_APPLY_FREE_SLOTS=0;" "BF_APPLY_FREE_SLOTS=1;" "BF_APPLY_FREE_SLOTS=2;" "BF_APPLY_FREE_SLOTS=1;--rehearse-shards 8" "BF_APPLY_FREE_SLOTS=2;--rehearse-shards 8" "BF_APPLY_FREE_SLOTS=0;"
# host side of the G = 8 rehearsal: HIP API calls per frame (counts exact; durations inflated by the tracer)
timeout -k 10 400 rocprofv3 --hip-trace --stats -d gpurun_out/$T/api -o api -- python3 bench.py --no-cpu-baseline --rehearse-shards 8 --steps 20 --warmup 5 > gpurun_out/$T/api.json 2> gpurun_out/$T/api.err || { echo "api trace failed"; tail -20 gpurun_out/$T/api.err; exit 1; }
f=$(find gpurun_out/$T/api -name "*hip_api_stats.csv" | head -1); [ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('hip api total %.1f ms' % (tot/1e6))
for r in rows[:25]: print('%-40s calls=%8s avg=%8.2fus total=%8.1fms' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
"
