#!/bin/bash
# Profiles of this round's loop: kernel trace of the bench (persistent PCG / cache / preprocessing
# timeline, tools/persist_gaps.py) and bench A/B of k_apply_ops mask variants (after their parity tests).
# Usage: tools/gpu_r8c.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/trace_bench.json 2> $O/trace_bench.err || { echo "trace run failed"; tail -20 $O/trace_bench.err; exit 1; }
python3 tools/persist_gaps.py $O/trace/run_kernel_trace.csv > $O/persist_gaps.txt 2>&1; cat $O/persist_gaps.txt
python3 tools/prof_summary.py $O/trace/run_kernel_stats.csv > $O/kernel_stats.txt && head -30 $O/kernel_stats.txt
gzip -f $O/trace/run_kernel_trace.csv
for v in qmask2 qmask1; do
  BF_HIP_LIB=$PWD/bundlefusion_amd/libbf_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_tsdf_gpu.py -x -q --timeout 300 --timeout-method thread -k "op_batch or fused" > $O/tests_$v.log 2>&1 || { echo "$v parity failed"; tail -30 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
for v in head qmask2 head qmask2 qmask1; do
  lib=""; [ $v != head ] && lib=$PWD/bundlefusion_amd/libbf_hip_$v.so
  BF_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/ab_$v.json 2> $O/ab_$v.err || { echo "bench $v failed"; tail -20 $O/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; pl=r['per_launch']; print('$v fps %.1f' % d['value'], 'apply_us %.1f' % r['avg_launch_us'], 'evals %.1fM upd %.1fM' % (pl['voxel_op_evaluations']/1e6, pl['voxel_op_updates']/1e6), 'gn_loop %.3f' % d['global_solve']['ms_per_gn_iter_in_loop'])"
done
