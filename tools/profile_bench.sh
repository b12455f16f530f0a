#!/bin/bash
# Kernel-time profile of the default bench command plus three PMC passes (FETCH_SIZE, WRITE_SIZE,
# SQ_INSTS_VALU) for the dominant kernel k_apply_ops (separate --pmc runs, kernel-trace only: no
# sys/runtime tracing with counters).
# Usage (on the GPU box): bash tools/profile_bench.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}; shift
OUT=gpurun_out/${TAG}
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $OUT/stats_bench.json 2> $OUT/stats_bench.err || { echo "stats pass failed"; tail -20 $OUT/stats_bench.err; exit 1; }
python3 tools/prof_summary.py $OUT/stats/run_kernel_stats.csv > $OUT/kernel_stats.txt && head -25 $OUT/kernel_stats.txt
rm -f $OUT/stats/run_kernel_trace.csv  # per-dispatch rows are large; the stats csv is what we keep
K=${PMC_KERNEL:-k_apply_ops}
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $OUT/fetch_bench.json 2> $OUT/fetch_bench.err || { echo "fetch pass failed"; tail -20 $OUT/fetch_bench.err; exit 1; }
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/write -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $OUT/write_bench.json 2> $OUT/write_bench.err || { echo "write pass failed"; tail -20 $OUT/write_bench.err; exit 1; }
timeout -k 10 500 rocprofv3 --pmc SQ_INSTS_VALU --kernel-include-regex "$K" -d $OUT/valu -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $OUT/valu_bench.json 2> $OUT/valu_bench.err || { echo "valu pass failed"; tail -20 $OUT/valu_bench.err; exit 1; }
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv "$K" $OUT/traffic.json $OUT/valu/run_counter_collection.csv
rm -rf $OUT/fetch $OUT/write $OUT/valu
