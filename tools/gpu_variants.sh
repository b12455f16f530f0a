#!/bin/bash
# A/B of voxel-pass variants on the GPU box: parity tests once, then the bench per env setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-var}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_tsdf_gpu.py tests/test_recon_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/${TAG}/pytest.log | head -20; tail -30 gpurun_out/${TAG}/pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}/pytest.log
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}/bench_$i.json 2> gpurun_out/${TAG}/bench_$i.err || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}/bench_$i.json')); print('$v', 'fps %.1f' % d['value'], 'apply_us %.1f' % d['roofline']['avg_launch_us'], 'integ_us %.1f' % d['roofline']['k_integrate']['avg_us'])"
done
