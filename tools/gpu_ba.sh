#!/bin/bash
# BA development loop on the GPU box: solver parity tests, standalone global-solve timing per mode,
# then the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-ba}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_recon_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
for m in 1 2; do
  BF_NORMAL_EQUATIONS=$m timeout -k 10 300 python -u tools/time_ba.py 500 > gpurun_out/${TAG}_time_ba_m$m.log 2>&1 || { echo "time_ba $m failed"; tail -20 gpurun_out/${TAG}_time_ba_m$m.log; exit 1; }
  echo "mode $m:"; tail -3 gpurun_out/${TAG}_time_ba_m$m.log
done
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo bench failed; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
