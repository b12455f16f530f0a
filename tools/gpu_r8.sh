#!/bin/bash
# Round-4 check: new tests first, the full GPU suite + smoke + default bench, then bench variants.
# Usage: tools/gpu_r8.sh TAG "pytest selectors" "variant args;variant args;..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; SEL=$2; VARS=$3
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest $SEL -x -v --timeout 300 --timeout-method thread > $O/first.log 2>&1 || { echo "first tests failed"; tail -40 $O/first.log; exit 1; }
  tail -1 $O/first.log
fi
if [ -z "$SKIP_SUITE" ]; then
  bash tools/gpu_check.sh $TAG || exit 1
fi
i=0
IFS=';' read -ra VA <<< "$VARS"
for v in "${VA[@]}"; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $v > $O/var$i.json 2> $O/var$i.err; rc=$?
  if [ $rc -ne 0 ]; then echo "variant $i ($v) rc=$rc"; tail -20 $O/var$i.err; exit 1; fi
  python3 -c "import json; d=json.load(open('$O/var$i.json')); r=d['roofline']; pl=r['per_launch']; print('var $i [$v]', 'fps %.1f' % d['value'], 'gn_ms %.3f loop %.3f' % (d['ms_per_gn_iter'], d['global_solve']['ms_per_gn_iter_in_loop']), 'apply_us %.1f' % r['avg_launch_us'], 'evals %.1fM upd %.1fM blocks %.0f ops %.2f' % (pl['voxel_op_evaluations']/1e6, pl['voxel_op_updates']/1e6, pl['work_list_blocks'], pl['ops']))"
done
