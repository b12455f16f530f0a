#!/bin/bash
# Kernel trace of a standalone global solve (tools/time_ba.py K) and the PCG launch analysis.
# Usage (GPU box): bash tools/profile_pcg.sh TAG [K]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; K=${2:-500}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/time_ba.py $K > $O/time_ba.txt 2> $O/time_ba.err || { tail -20 $O/time_ba.err; exit 1; }
cat $O/time_ba.txt
python3 tools/pcg_standalone.py $(ls $O/trace/*/run_kernel_trace.csv 2>/dev/null || ls $O/trace/run_kernel_trace.csv) | tee $O/pcg_launches.txt
python3 tools/prof_summary.py $(ls $O/trace/*/run_kernel_stats.csv 2>/dev/null || ls $O/trace/run_kernel_stats.csv) > $O/kernel_stats.txt; head -12 $O/kernel_stats.txt
rm -f $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv
