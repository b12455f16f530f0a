cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=bundlefusion_amd; mkdir -p gpurun_out
BF_HIP_LIB=$PWD/$L/libbf_hip_projpk.so timeout -k 10 600 python -u -m pytest tests/test_tsdf_gpu.py tests/test_recon_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r7f_projpk_tests.log 2>&1 || { tail -30 gpurun_out/r7f_projpk_tests.log; exit 1; }
tail -1 gpurun_out/r7f_projpk_tests.log
SKIP_TESTS=1 bash tools/gpu_abn.sh r7f "cur projpk=$L/libbf_hip_projpk.so cur projpk=$L/libbf_hip_projpk.so" --steps 20 --warmup 5
