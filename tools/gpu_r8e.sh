#!/bin/bash
# changed GPU tests, then bench A/B (preprocessing wait placement), bench variants, a G = 8 rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_recon_gpu.py tests/test_ba_gpu.py tests/test_recon_parity_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
summ() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; pl=r['per_launch']; print('$2', 'fps %.1f' % d['value'], 'apply_us %.1f' % r['avg_launch_us'], 'evals %.3fM upd %.3fM blocks %.1f' % (pl['voxel_op_evaluations']/1e6, pl['voxel_op_updates']/1e6, pl['work_list_blocks']), 'gn %.3f loop %.3f' % (d['ms_per_gn_iter'], d['global_solve']['ms_per_gn_iter_in_loop']), 'rc_us %.1f' % d['raycast']['k_render_us'], 'rc_frac %.3f' % d['raycast']['roofline']['frac'])"; }
i=0
for v in "new" "early" "new" "early" "new --no-preprocess" "new --result-lag 0" "new --rehearse-shards 8"; do
  i=$((i+1)); name=${v%% *}; args=""; [ "$v" != "$name" ] && args=${v#* }
  lib=""; [ $name != new ] && lib=$PWD/bundlefusion_amd/libbf_hip_$name.so
  BF_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 $args > $O/b$i.json 2> $O/b$i.err || { echo "bench $v failed"; tail -20 $O/b$i.err; exit 1; }
  summ $O/b$i.json "$i [$v]"
done
