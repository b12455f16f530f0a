#!/bin/bash
# after the priority policy: loop tests, the driver's bench (with the CPU baseline, as the driver runs it),
# the default bench, config 4's 20k-frame stream (default priority there)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_recon_gpu.py tests/test_recon_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_bench.json 2> $O/driver_bench.err || { echo "driver bench failed"; tail -20 $O/driver_bench.err; exit 1; }
timeout -k 10 600 python -u bench.py > $O/default_bench.json 2> $O/default_bench.err || { echo "default bench failed"; tail -20 $O/default_bench.err; exit 1; }
for f in driver_bench default_bench; do python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=d['roofline']; l=d['loop']; print('$f fps %.1f' % d['value'], 'apply_us %.1f frac %.3f' % (r['avg_launch_us'], r['frac']), 'traffic', r['traffic'] is not None, 'valu', r['valu'] is not None, 'gn %.3f loop %.3f' % (d['ms_per_gn_iter'], d['global_solve']['ms_per_gn_iter_in_loop']), 'host %.0f wait %.0f' % (1e3*l['host_ms_per_frame'], 1e3*l['host_wait_ms_per_frame']))"; done
bash tools/gpu_lag.sh $T "--frames 20000" "--rehearse-shards 8"
