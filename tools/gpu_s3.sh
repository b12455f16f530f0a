set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s3_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/s3_pytest.log; exit 1; }
tail -5 gpurun_out/s3_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_smoke.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/s3_smoke.log; exit 1; }
tail -2 gpurun_out/s3_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s3_bench.json 2> gpurun_out/s3_bench.err || { echo bench failed; tail -30 gpurun_out/s3_bench.err; exit 1; }
cat gpurun_out/s3_bench.json
