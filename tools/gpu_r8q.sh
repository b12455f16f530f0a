#!/bin/bash
# host time per loop section (BF_HOST_PROFILE build) at N = 1 and in the G = 8 rehearsal; config 5 and
# config 4's 20 000-frame stream on the current code
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
bash tools/gpu_envab.sh $T "BF_HIP_LIB=bundlefusion_amd/libbf_hip_hostprof.so;--rehearse-shards 8" "BF_HIP_LIB=bundlefusion_amd/libbf_hip_hostprof.so;--rehearse-shards 8 --async-bundling 2" "BF_HIP_LIB=bundlefusion_amd/libbf_hip_hostprof.so;" || exit 1
grep -h "host us per frame" gpurun_out/$T/e*.err
bash tools/gpu_configs.sh $T
