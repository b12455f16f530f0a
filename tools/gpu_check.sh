#!/bin/bash
# Full GPU check: the -m gpu suite, smoke(), and the default bench line. Usage: tools/gpu_check.sh TAG [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-check}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/$TAG/pytest.log | head -20; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo bench failed; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench.json')); r=d['roofline']; pl=r['per_launch']; print('fps %.1f' % d['value'], 'gn_ms %.3f' % d['ms_per_gn_iter'], 'apply_us %.1f' % r['avg_launch_us'], 'evals %.1fM upd %.1fM blocks %.0f ops %.1f' % (pl['voxel_op_evaluations']/1e6, pl['voxel_op_updates']/1e6, pl['work_list_blocks'], pl['ops']), 'frac %.3f' % r['frac'])"
