cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=bundlefusion_amd; mkdir -p gpurun_out
SKIP_TESTS=1 bash tools/gpu_abn.sh r7i "cur split=$L/libbf_hip_split.so split7=$L/libbf_hip_split7.so cur split=$L/libbf_hip_split.so split7=$L/libbf_hip_split7.so" --steps 20 --warmup 5
timeout -k 10 400 python -u bench.py --no-cpu-baseline --rehearse-shards 8 --steps 20 --warmup 5 > gpurun_out/r7i/rehearse_g8.json 2> gpurun_out/r7i/rehearse_g8.err || { tail -20 gpurun_out/r7i/rehearse_g8.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r7i/rehearse_g8.json').read().strip().splitlines()[-1]); print('rehearse g8 fps %.1f' % d['value'], 'gn_loop_ms %.3f' % d['global_solve']['ms_per_gn_iter_in_loop'])"
