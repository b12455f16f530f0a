#!/bin/bash
# round-2 pass d: local verification + loop-level parity tests, then the whole GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r2d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_verify_gpu.py tests/test_recon_parity_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1 || { echo "new tests failed"; tail -60 $O/pytest_new.log; exit 1; }
grep -E "passed|failed|max diff|end dense" $O/pytest_new.log | tail -5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || { echo "suite failed"; tail -40 $O/pytest_all.log; exit 1; }
tail -2 $O/pytest_all.log
