#!/bin/bash
# One GPU call: the -m gpu suite on the current library (unless SKIP_TESTS=1), then bench runs of
# library variants in the given order (A/B/A/B...). A variant is NAME or NAME=LIB (LIB relative to the
# repo; NAME alone = the in-tree libbf_hip.so). Stops at the first step that times out, faults or aborts.
# Usage: tools/gpu_abn.sh TAG "head=bundlefusion_amd/libbf_hip_head.so new head=... new" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; V=${2:-}; shift 2
mkdir -p $O
run() {  # log name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2> $O/$n.err; local rc=$?
  echo "$n rc=$rc: $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then tail -30 $O/$n.err; tail -30 $O/$n.log; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  run gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
i=0
for v in $V; do
  i=$((i + 1))
  name=${v%%=*}; lib=""; [ "$v" != "$name" ] && lib=${v#*=}
  BF_HIP_LIB=${lib:+$PWD/$lib} run bench_${i}_$name 400 python -u bench.py --no-cpu-baseline "$@"
  python3 -c "import json; d=json.loads(open('$O/bench_${i}_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', 'fps %.1f' % d['value'], 'apply_us %.1f' % r['avg_launch_us'], 'gn_ms %.3f' % d['ms_per_gn_iter'], 'gn_loop_ms %.3f' % d['global_solve']['ms_per_gn_iter_in_loop'], 'evals %.1fM' % (r['per_launch']['voxel_op_evaluations'] / 1e6))"
done
