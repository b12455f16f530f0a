#!/bin/bash
# One extra bench run for an A/B comparison (set the variant's env vars on the command line).
# Usage: VAR=... tools/gpu_ab.sh TAG NAME [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-ab}; NAME=${2:-b}; shift 2
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/$TAG/bench_$NAME.json 2> gpurun_out/$TAG/bench_$NAME.err || { echo "bench $NAME failed"; tail -30 gpurun_out/$TAG/bench_$NAME.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$NAME.json')); r=d['roofline']; print('$NAME fps %.1f' % d['value'], 'apply_us %.1f' % r['avg_launch_us'])"
