set -o pipefail
D=gpurun_out/$1; shift
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_tsdf_gpu.py tests/test_recon_gpu.py -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline > $D/b.json 2>$D/b.err || { tail $D/b.err; exit 1; }
  echo "$cfg $(grep -o '"value": [0-9.]*\|avg_launch_us": [0-9.]*' $D/b.json | tr '\n' ' ')"
done
