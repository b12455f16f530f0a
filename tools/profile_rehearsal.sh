#!/bin/bash
# Kernel-time profile of one rank's share of a G-way TSDF-sharded run (bench.py --rehearse-shards G),
# for G in the given list: what each rank's scene stream costs per frame without G GPUs.
# Usage (on the GPU box): bash tools/profile_rehearsal.sh TAG "2 8" [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; GS=$2; shift 2
OUT=gpurun_out/${TAG}
mkdir -p $OUT
for G in $GS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/g$G -o run --output-format csv -- python3 bench.py --no-cpu-baseline --rehearse-shards $G "$@" > $OUT/bench_g$G.json 2> $OUT/bench_g$G.err || { echo "G=$G failed"; tail -20 $OUT/bench_g$G.err; exit 1; }
  python3 tools/prof_summary.py $OUT/g$G/run_kernel_stats.csv > $OUT/kernel_stats_g$G.txt
  rm -f $OUT/g$G/run_kernel_trace.csv
  echo "G=$G: $(python3 -c "import json; d=json.loads(open('$OUT/bench_g$G.json').read().strip().splitlines()[-1]); print('%.1f frames/s' % d['value'], d['config']['parallelism'])")"
  head -8 $OUT/kernel_stats_g$G.txt
done
