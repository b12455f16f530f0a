#!/bin/bash
# TSDF development loop on the GPU box: scene parity tests, bench, SQ_INSTS_VALU of k_apply_ops.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-tsdf}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_tsdf_gpu.py tests/test_recon_gpu.py tests/test_raycast_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/${TAG}/pytest.log | head -20; tail -30 gpurun_out/${TAG}/pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}/pytest.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}/bench.json 2> gpurun_out/${TAG}/bench.err || { echo bench failed; tail -30 gpurun_out/${TAG}/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}/bench.json')); print('value', d['value'], 'apply_us', d['roofline']['avg_launch_us'], 'evals', d['roofline']['per_launch']['voxel_op_evaluations'], 'ms_gn', d['ms_per_gn_iter'])"
timeout -k 10 500 rocprofv3 --pmc SQ_INSTS_VALU --kernel-include-regex k_apply_ops -d gpurun_out/$TAG/valu -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/$TAG/valu_bench.json 2> gpurun_out/$TAG/valu_bench.err || { echo "valu pass failed"; tail -20 gpurun_out/$TAG/valu_bench.err; exit 1; }
python3 - <<PY
import csv, glob
rows = list(csv.DictReader(open(glob.glob('gpurun_out/$TAG/valu/**/run_counter_collection.csv', recursive=True)[0])))
v = [float(r['Counter_Value']) for r in rows if r.get('Counter_Name') == 'SQ_INSTS_VALU']
print('SQ_INSTS_VALU per k_apply_ops launch:', sum(v) / max(1, len(set(r['Dispatch_Id'] for r in rows))), 'dispatches', len(set(r['Dispatch_Id'] for r in rows)))
PY
