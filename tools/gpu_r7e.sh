cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile_bench.sh r7e_s50 || exit 1
bash tools/profile_bench.sh r7e_s20 --steps 20 --warmup 5
