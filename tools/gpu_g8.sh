#!/bin/bash
# G = 8 rehearsal diagnosis: with / without in-loop preprocessing, and a kernel trace (GPU busy fraction)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O; shift
bash tools/gpu_lag.sh $1 "--rehearse-shards 8 --result-lag 20 --no-preprocess" "--rehearse-shards 8 --result-lag 20" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --rehearse-shards 8 --result-lag 20 > $O/trace_bench.json 2> $O/trace_bench.err || { echo "trace failed"; tail -20 $O/trace_bench.err; exit 1; }
python3 tools/gpu_busy.py $O/trace/run_kernel_trace.csv 4800 200
gzip -f $O/trace/run_kernel_trace.csv
