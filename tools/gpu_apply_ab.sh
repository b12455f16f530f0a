#!/bin/bash
# A/B of the op-batch voxel-pass variants (BF_APPLY_ZIN): op-batch parity tests, then the bench's
# k_apply_ops launch time, per variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p $O
for V in ${VARIANTS:-0 4 2}; do
  BF_APPLY_ZIN=$V timeout -k 10 300 python -u -m pytest tests/test_tsdf_gpu.py tests/test_recon_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batch or reintegrate or replay" > $O/pytest_$V.log 2>&1 || { echo "variant $V parity failed"; tail -30 $O/pytest_$V.log; exit 1; }
  BF_APPLY_ZIN=$V timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$V.json 2> $O/bench_$V.err || { echo "variant $V bench failed"; tail -20 $O/bench_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$V.json')); r=d['roofline']; print('variant $V', 'fps %.1f' % d['value'], 'apply_us %.1f' % r['avg_launch_us'], '$(tail -1 $O/pytest_$V.log)')"
done
