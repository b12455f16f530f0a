set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/$1; shift
mkdir -p $D
for cfg in "$@"; do
  env $cfg timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/st -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 > $D/b.json 2>$D/b.err || { tail $D/b.err; exit 1; }
  echo "== $cfg"; python3 tools/prof_summary.py $D/st/run_kernel_stats.csv | grep -E "$PROF_RX"
  rm -rf $D/st
done
