#!/bin/bash
# Kernel-time profile of the bench command plus three PMC passes (FETCH_SIZE, WRITE_SIZE,
# SQ_INSTS_VALU) for the dominant kernel k_apply_ops (separate --pmc runs, kernel-trace only: no
# sys/runtime tracing with counters). The PMC figures are averaged over the bench's timed launches
# and tagged with its workload string (tools/pmc_traffic.py --bench).
# Usage (on the GPU box): bash tools/profile_bench.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}; shift
OUT=gpurun_out/${TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $OUT/stats_bench.json 2> $OUT/stats_bench.err || { echo "stats pass failed"; tail -20 $OUT/stats_bench.err; exit 1; }
python3 tools/prof_summary.py $OUT/stats/run_kernel_stats.csv > $OUT/kernel_stats.txt && head -25 $OUT/kernel_stats.txt
# the dominant kernel over the bench's timed region only (its last roofline.launches dispatches): the figure
# the bench line's avg_launch_us (HIP events) must agree with; the stats csv averages the whole stream
python3 - $OUT/stats/run_kernel_trace.csv $OUT/stats_bench.json > $OUT/apply_timed_region.txt <<'PY'
import csv, json, sys
sys.path.insert(0, "tools")
from timed_region import bench_counts, window
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
n, after = bench_counts(sys.argv[2])
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_apply_ops" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = window(rows, n, after)
us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in last]
print("k_apply_ops over the timed region (%d of %d dispatches, before the end phase's %d): avg %.1f us (rocprofv3 kernel "
      "trace); the profiled bench line's HIP-event average %.1f us" % (len(us), len(rows), after, sum(us) / max(1, len(us)),
                                                                       d["roofline"]["avg_launch_us"]))
PY
cat $OUT/apply_timed_region.txt
rm -f $OUT/stats/run_kernel_trace.csv  # per-dispatch rows are large; the stats csv is what we keep
K=${PMC_KERNEL:-k_apply_ops}
for C in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$K" -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $OUT/pmc_${C}_bench.json 2> $OUT/pmc_${C}_bench.err || { echo "$C pass failed"; tail -20 $OUT/pmc_${C}_bench.err; exit 1; }
done
python3 tools/pmc_traffic.py $OUT/pmc_FETCH_SIZE/run_counter_collection.csv $OUT/pmc_WRITE_SIZE/run_counter_collection.csv "$K" $OUT/traffic.json $OUT/pmc_SQ_INSTS_VALU/run_counter_collection.csv --bench $OUT/pmc_FETCH_SIZE_bench.json
rm -rf $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $OUT/pmc_SQ_INSTS_VALU
