#!/bin/bash
# standalone preprocessing / cache kernel times; HIP API calls per frame of the G = 8 rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/pre -o pre --output-format csv -- python3 tools/time_preproc.py 300 > gpurun_out/$T/pre.log 2>&1 || { echo "time_preproc failed"; tail -20 gpurun_out/$T/pre.log; exit 1; }
grep "us/frame" gpurun_out/$T/pre.log
f=$(find gpurun_out/$T/pre -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 tools/prof_summary.py $f > gpurun_out/$T/pre_kernels.txt; cat gpurun_out/$T/pre_kernels.txt
find gpurun_out/$T/pre -name "*trace.csv" -delete
# host side of the G = 8 rehearsal: HIP API calls per frame (counts exact; durations inflated by the tracer)
timeout -k 10 400 rocprofv3 --hip-trace --stats -d gpurun_out/$T/api -o api --output-format csv -- python3 bench.py --no-cpu-baseline --rehearse-shards 8 --steps 20 --warmup 5 > gpurun_out/$T/api.json 2> gpurun_out/$T/api.err || { echo "api trace failed"; tail -20 gpurun_out/$T/api.err; exit 1; }
f=$(find gpurun_out/$T/api -name "*hip_api_stats.csv" | head -1)
[ -n "$f" ] || { echo "no api stats"; find gpurun_out/$T/api | head; exit 1; }
python3 - "$f" > gpurun_out/$T/api_summary.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('hip api total %.1f ms over %d calls' % (tot / 1e6, sum(int(r['Calls']) for r in rows)))
for r in rows[:40]:
    print('%-44s calls=%8s avg=%8.2fus total=%8.1fms' % (r['Name'][:44], r['Calls'], float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e6))
PY
cat gpurun_out/$T/api_summary.txt
find gpurun_out/$T/api -name "*trace.csv" -delete
tail -c 600 gpurun_out/$T/api.json
