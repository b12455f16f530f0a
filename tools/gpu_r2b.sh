#!/bin/bash
# round-2 pass b: new BA parity tests + scan with fixed schedules + bench profile (traffic of the driver workload)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r2b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "bench_scale or fixed_schedule" > $O/pytest_ba.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_ba.log; }
tail -3 $O/pytest_ba.log
timeout -k 10 400 python3 -u tools/ba_parity_scan.py > $O/ba_scan.log 2>&1 || { echo "scan failed"; tail -20 $O/ba_scan.log; exit 1; }
bash tools/profile_bench.sh r2b_prof --steps 20 --warmup 5 || exit 1
echo done
