#!/bin/bash
# round-2 first GPU pass: host info, GPU tests, the driver's bench command, BA parity scan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r2a; mkdir -p $O
{ nproc; grep -m1 "model name" /proc/cpuinfo; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; grep -m1 flags /proc/cpuinfo | tr ' ' '\n' | grep -E "^(avx512f|avx2|fma)$"; } > $O/host.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python3 -u tools/ba_parity_scan.py > $O/ba_scan.log 2>&1 || { echo "scan failed"; tail -20 $O/ba_scan.log; exit 1; }
echo done
