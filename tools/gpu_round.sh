#!/bin/bash
# One GPU call: the large-scene test, the GPU suite, then bench A/B runs of k_apply_ops variants.
# Stops at the first step that times out, faults or aborts (exit status > 1).
# Usage: bash tools/gpu_round.sh TAG "VARIANTS" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; V=${2:-}; shift 2
mkdir -p $O
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc: $(tail -1 $O/$n.log)"
  if [ $rc -gt 1 ]; then tail -30 $O/$n.log; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  run gpu 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_large_scene_gpu.py::test_config5_frames_parity_and_beyond_2_22_blocks
fi
for v in $V; do
  run bench_$v 300 python -u bench.py --no-cpu-baseline "$@"
  python3 -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('variant $v', 'fps %.1f' % d['value'], 'apply_us %.1f' % r['avg_launch_us'], 'gn_ms %.3f' % d['ms_per_gn_iter'], 'gn_loop_ms %.3f' % d['global_solve']['ms_per_gn_iter_in_loop'], 'dense_end_ms %.2f' % d['global_dense_end_solve']['ms'], 'evals %.1fM' % (r['per_launch']['voxel_op_evaluations'] / 1e6), 'blocks %.0fk' % (r['per_launch']['work_list_blocks'] / 1e3))"
done
if [ -z "$SKIP_LARGE" ]; then
  run large 300 python -u -m pytest -s tests/test_large_scene_gpu.py -x -v --timeout 280 --timeout-method thread
fi
