#!/bin/bash
# SQ counters of one kernel of the bench (separate --pmc pass, kernel-trace only).
# Usage: bash tools/gpu_sqpmc.sh TAG KERNEL_REGEX "COUNTERS..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; K=$2; CNT=$3; shift 3
mkdir -p gpurun_out/$TAG
timeout -s KILL 300 rocprofv3 --pmc $CNT --kernel-include-regex "$K" -d gpurun_out/$TAG/pmc -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 60 "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "pmc pass failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 - <<PY
import csv, glob, collections
f = glob.glob('gpurun_out/$TAG/pmc/**/run_counter_collection.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
acc = collections.defaultdict(float); disp = set()
for r in rows:
    acc[r['Counter_Name']] += float(r['Counter_Value']); disp.add(r['Dispatch_Id'])
n = max(1, len(disp))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {v / n:16.1f} per dispatch  ({n} dispatches)")
PY
