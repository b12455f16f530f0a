#!/bin/bash
# bench A/B over environment settings: each argument is "ENV_ASSIGNMENTS;BENCH_FLAGS"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O; shift
summ() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; pl=r['per_launch']; l=d['loop']; print('$2', 'host %.0f wait %.0f us' % (1e3*l.get('host_ms_per_frame',0), 1e3*l.get('host_wait_ms_per_frame',0)), 'fps %.1f' % d['value'], 'apply_us %.1f' % r['avg_launch_us'], 'evals/upd %.3f' % (pl['voxel_op_evaluations']/max(1,pl['voxel_op_updates'])), 'gn %.3f loop %.3f' % (d['ms_per_gn_iter'], d['global_solve']['ms_per_gn_iter_in_loop']), 'local_ms %.2f global_ms %.2f' % (l['local_solve_ms'], l['global_solve_ms']))"; }
i=0
for v in "$@"; do
  i=$((i+1))
  e=${v%%;*}; f=${v#*;}
  env $e timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 $f > $O/e$i.json 2> $O/e$i.err || { echo "bench [$v] failed"; tail -20 $O/e$i.err; exit 1; }
  summ $O/e$i.json "$i [$v]"
done
