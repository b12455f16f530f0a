#!/bin/bash
# Bench lines of the other BASELINE shapes on one GPU: config 5 (1280x960 at 2 mm) and config 4's
# 20 000-frame stream (2 001 keyframes). Usage: tools/gpu_configs.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python -u bench.py --no-cpu-baseline --preset config5 --steps 20 --warmup 5 > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/config5.json').read().strip().splitlines()[-1]); print('config5 fps %.1f' % d['value'], 'whole %.1f' % d['stream']['frames_per_s_whole_stream'], 'apply_us %.1f' % d['roofline']['avg_launch_us'], 'frac %.3f' % d['roofline']['frac'])"
timeout -k 10 600 python -u bench.py --no-cpu-baseline --frames 20000 --steps 20 --warmup 5 > $O/stream20k.json 2> $O/stream20k.err || { tail -20 $O/stream20k.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/stream20k.json').read().strip().splitlines()[-1]); print('20k fps %.1f' % d['value'], 'whole %.1f' % d['stream']['frames_per_s_whole_stream'], 'gn_ms %.3f' % d['ms_per_gn_iter'], 'gn_loop_ms %.3f' % d['global_solve']['ms_per_gn_iter_in_loop'], 'K', d['global_solve']['keyframes'])"
