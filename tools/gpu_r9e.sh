#!/bin/bash
# kernel trace of the driver workload: how much of the preprocessing / cache kernels' in-loop intervals the
# voxel pass covers (slot waits), next to their standalone times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "trace failed"; tail -20 $O/bench.err; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 tools/overlap_attr.py $f 200 > $O/overlap.txt; cat $O/overlap.txt
rm -f $f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pre -o pre --output-format csv -- python3 tools/time_preproc.py 300 > $O/pre.log 2>&1 || { echo "time_preproc failed"; tail -20 $O/pre.log; exit 1; }
python3 tools/prof_summary.py $O/pre/pre_kernel_stats.csv | head -6
find $O/pre -name "*trace.csv" -delete
