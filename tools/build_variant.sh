#!/bin/bash
# Builds bundlefusion_amd/libbf_hip_<NAME>.so: the library with one source (tsdf by default, or ba,
# ...) compiled under extra defines (kernel variants and measurement builds for an A/B timing run:
# the ab: step of tools/gpu.sh). Usage: tools/build_variant.sh NAME "-DBF_APPLY_ZC=2 ..." [SRC]
# (after `make -C bundlefusion_amd/csrc`)
set -e
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2; SRC=${3:-tsdf}
OBJ=build/hip/${SRC}_var_$NAME.o
F=bundlefusion_amd/csrc/$SRC.hip; [ -f $F ] || F=bundlefusion_amd/csrc/$SRC.cpp
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -munsafe-fp-atomics $DEFS -x hip -c $F -o $OBJ
OBJS=$(ls build/hip/*.o | grep -v "/${SRC}[._]" | grep -v "_var_\|_rev_")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib -lz -o bundlefusion_amd/libbf_hip_$NAME.so $OBJS $OBJ -L/opt/rocm/lib -lrccl
echo bundlefusion_amd/libbf_hip_$NAME.so
