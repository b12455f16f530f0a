#!/bin/bash
# one default bench line (the driver's command) into gpurun_out/TAG/bench.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-bench}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo bench failed; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); r=d['roofline']; c=d.get('cpu_baseline',{})
print('fps %.1f' % d['value'], 'gn_ms %.3f' % d['ms_per_gn_iter'], 'apply_us %.1f' % r['avg_launch_us'], 'frac %.3f' % r['frac'])
print('dense end', json.dumps(d['global_dense_end_solve']))
print('cpu', c.get('value'), c.get('steady_state_frames_per_s'), c.get('gpu_prefix_frames_per_s'), json.dumps(c.get('loop_prefix')))
"
