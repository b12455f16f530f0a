cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; O=gpurun_out/r7c; mkdir -p $O
P=$PWD/bundlefusion_amd/libbf_hip_ptag.so
BF_HIP_LIB=$P timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 300 --timeout-method thread > $O/ba_ptag.log 2>&1 || { tail -30 $O/ba_ptag.log; exit 1; }
tail -1 $O/ba_ptag.log
for L in cur ptag cur ptag; do
  if [ $L = ptag ]; then export BF_HIP_LIB=$P; else unset BF_HIP_LIB; fi
  timeout -k 10 300 python -u tools/time_ba.py 500 > $O/time_$L.log 2>&1 || { tail -20 $O/time_$L.log; exit 1; }
  echo "$L $(tail -1 $O/time_$L.log | cut -c1-300)"
done
unset BF_HIP_LIB
SKIP_TESTS=1 bash tools/gpu_abn.sh r7c "cur ptag=bundlefusion_amd/libbf_hip_ptag.so cur ptag=bundlefusion_amd/libbf_hip_ptag.so" --steps 20 --warmup 5
