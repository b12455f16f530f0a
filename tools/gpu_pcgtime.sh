#!/bin/bash
# per-phase timings of the persistent PCG (BF_PCG_TIMING build) at K = 500 and K = 2 001, standalone
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for K in 500 2001; do
  BF_HIP_LIB=$PWD/bundlefusion_amd/libbf_hip_pcgtime.so timeout -k 10 300 python3 tools/time_ba.py $K > $O/pcgtime_$K.txt 2>&1 || { echo "K=$K failed"; tail -20 $O/pcgtime_$K.txt; exit 1; }
  grep -E "persistent pcg|finisher|workers|ms_per_gn" $O/pcgtime_$K.txt | head -8
  timeout -k 10 300 python3 tools/time_ba.py $K > $O/time_$K.txt 2>&1 || exit 1
  tail -1 $O/time_$K.txt
done
