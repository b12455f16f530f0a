#!/bin/bash
# Builds bundlefusion_amd/libbf_hip_<NAME>.so with one source (tsdf.hip by default, or ba, ...) taken
# from git revision REV (the other objects from the current build): the A/B baseline of a kernel change
# (the ab: step of tools/gpu.sh). Usage: tools/build_rev.sh REV NAME [SRC]
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2; BASE=${3:-tsdf}
SRC=bundlefusion_amd/csrc/${BASE}_rev_$NAME.hip
git show $REV:bundlefusion_amd/csrc/$BASE.hip > $SRC
trap 'rm -f $SRC' EXIT
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -munsafe-fp-atomics -x hip -c $SRC -o build/hip/${BASE}_rev_$NAME.o
OBJS=$(ls build/hip/*.o | grep -v "/${BASE}[._]" | grep -v "_var_\|_rev_")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib -lz -o bundlefusion_amd/libbf_hip_$NAME.so $OBJS build/hip/${BASE}_rev_$NAME.o -L/opt/rocm/lib -lrccl
echo bundlefusion_amd/libbf_hip_$NAME.so
