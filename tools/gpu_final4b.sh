#!/bin/bash
# Round-4 last check on HEAD: the -m gpu suite, smoke, the driver's bench, the default bench, G = 8 rehearsal,
# config 5 (10 000 frames) and config 4's 20 000-frame stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_check.sh $T --gpus 1 --steps 20 --warmup 5 || exit 1
timeout -k 10 600 python -u bench.py > $O/default_bench.json 2> $O/default_bench.err || { echo "default bench failed"; tail -20 $O/default_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/default_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('default fps %.1f' % d['value'], 'traffic', r['traffic'] is not None, 'valu', r['valu'] is not None)"
bash tools/gpu_lag.sh $T "--rehearse-shards 8" "--preset config5" "--frames 20000" || exit 1
