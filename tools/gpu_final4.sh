#!/bin/bash
# Round-4 final check on HEAD: the -m gpu suite, smoke, the driver's bench (--steps 20 --warmup 5) and the
# default bench (no flags), config 5 at BASELINE's 10 000 frames, G = 8 rehearsal with result lags 20 / 30
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_check.sh $T --gpus 1 --steps 20 --warmup 5 || exit 1
timeout -k 10 600 python -u bench.py > $O/default_bench.json 2> $O/default_bench.err || { echo "default bench failed"; tail -20 $O/default_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/default_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('default fps %.1f' % d['value'], 'traffic', r['traffic'] is not None, 'valu', r['valu'] is not None)"
bash tools/gpu_lag.sh $T "--rehearse-shards 8" "--rehearse-shards 8 --result-lag 30" || exit 1
timeout -k 10 700 python -u bench.py --no-cpu-baseline --preset config5 --frames 10000 --steps 20 --warmup 5 > $O/config5_10k.json 2> $O/config5_10k.err || { echo "config5 10k failed"; tail -20 $O/config5_10k.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/config5_10k.json').read().strip().splitlines()[-1]); print('config5 10k fps %.1f' % d['value'], 'whole %.1f' % d['stream']['frames_per_s_whole_stream'], 'apply_us %.1f' % d['roofline']['avg_launch_us'], 'gn %.3f loop %.3f' % (d['ms_per_gn_iter'], d['global_solve']['ms_per_gn_iter_in_loop']), 'K', d['global_solve']['keyframes'])"
