#!/bin/bash
# One GPU call made of named steps, run in order; each step has its own time limit and the call stops at
# the first step that times out, faults or aborts (exit status > 1; a failing test, status 1, goes on).
# Outputs go to gpurun_out/TAG/. Usage: bash tools/gpu.sh TAG STEP [STEP ...]; in ARGS, ',' stands for ' '.
#   tests[:EXPR]           pytest -m gpu [-k EXPR]
#   test:PATH[:EXPR]       pytest one file (node ids allowed) [-k EXPR]
#   smoke                  __graft_entry__.smoke()
#   bench:NAME[:ARGS]      python bench.py --no-cpu-baseline ARGS            -> bench_NAME.json
#   fullbench:NAME[:ARGS]  python bench.py ARGS (with the CPU baseline)      -> bench_NAME.json
#   ab:LIB:NAME[:ARGS]     the bench with BF_HIP_LIB=bundlefusion_amd/libbf_hip_LIB.so (a variant build)
#   envbench:NAME:VAR=VAL[+VAR=VAL...][:ARGS]  the bench with environment settings (runtime A/B switches)
#   env:VAR=VAL[+...] / unenv:VAR[+...]  set / clear environment settings for the steps that follow
#   profile:NAME[:ARGS]    tools/profile_bench.sh TAG/NAME ARGS (kernel stats + FETCH/WRITE/VALU passes)
#   sqpmc:NAME:KERNEL:CNT[:ARGS]  one --pmc pass of counters CNT (',' separated) over KERNEL's dispatches
#   sens:N[:ARGS]          write an N-frame synthetic .sens (tools/make_sens.py), then bench.py --sens ARGS
#   trace:NAME[:ARGS]      kernel trace of the bench (rocprofv3 --kernel-trace): the scene stream's per-frame timeline
#                          (tools/stream_timeline.py) and the input kernels' overlap with the voxel pass (overlap_attr.py)
#   py:NAME:SECONDS:ARGS   python ARGS (a tool script) with a SECONDS limit -> NAME.log
#   avail                  the counters rocprofv3 offers on this GPU -> avail.log
#   kstats:NAME[:ARGS]     rocprofv3 --kernel-trace --stats of the bench -> kstats_NAME.csv (per-kernel summary)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  echo "[$(date +%T)] $n: $*"
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$(date +%T)] $n rc=$rc: $(tail -1 $O/$n.log | cut -c1-400)"
  if [ $rc -gt 1 ]; then tail -40 $O/$n.log; exit $rc; fi
  return 0
}
summ() {  # one line of a bench JSON
  python3 - "$1" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
except Exception as e:
    print("no bench line:", e); sys.exit(0)
r = d.get("roofline") or {}
pl = r.get("per_launch") or {}
print("fps %.1f" % d["value"], "apply_us %.1f" % r.get("avg_launch_us", 0), "gn_ms %s" % d.get("ms_per_gn_iter"),
      "gn_loop_ms %s" % (d.get("global_solve") or {}).get("ms_per_gn_iter_in_loop"),
      "evals %.1fM" % (pl.get("voxel_op_evaluations", 0) / 1e6), "blocks %.0fk" % (pl.get("work_list_blocks", 0) / 1e3),
      "host %s" % json.dumps(d.get("host")) if "host" in d else "")
PY
}
for step in "$@"; do
  IFS=: read -r kind a b c d <<< "$step"
  case $kind in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${a:+-k "${a//,/ }"} ;;
    test) run "test_$(basename ${a%%.py*})" 900 python -u -m pytest -s "$a" -x -v --timeout 600 --timeout-method thread ${b:+-k "${b//,/ }"} ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench_$a 900 python -u bench.py --no-cpu-baseline ${b//,/ }; cp $O/bench_$a.log $O/bench_$a.json; summ $O/bench_$a.json ;;
    fullbench) run bench_$a 900 python -u bench.py ${b//,/ }; cp $O/bench_$a.log $O/bench_$a.json; summ $O/bench_$a.json ;;
    ab) BF_HIP_LIB=bundlefusion_amd/libbf_hip_$a.so run bench_$b 900 python -u bench.py --no-cpu-baseline ${c//,/ }; summ $O/bench_$b.log ;;
    env) IFS=+ read -ra KV <<< "$a"; for x in "${KV[@]}"; do export "$x"; done; echo "[env] $a" ;;
    unenv) IFS=+ read -ra KV <<< "$a"; for x in "${KV[@]}"; do unset "${x%%=*}"; done; echo "[unenv] $a" ;;
    envbench) IFS=+ read -ra KV <<< "$b"; for x in "${KV[@]}"; do export "$x"; done
              run bench_$a 900 python -u bench.py --no-cpu-baseline ${c//,/ }; for x in "${KV[@]}"; do unset "${x%%=*}"; done; summ $O/bench_$a.log ;;
    profile) run profile_$a 1100 bash tools/profile_bench.sh $TAG/$a ${b//,/ } ;;
    sqpmc) run sqpmc_$a 300 rocprofv3 --pmc ${c//,/ } --kernel-include-regex "$b" -d $O/sqpmc_$a -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${d//,/ }
           python3 tools/pmc_kernel.py "$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0])" $O/sqpmc_$a)" "$b" > $O/sqpmc_$a.txt; cat $O/sqpmc_$a.txt; rm -rf $O/sqpmc_$a ;;
    sens) run make_sens_$a 900 python -u tools/make_sens.py $a /tmp/synthetic_$a.sens
          run sens_$a 1100 python -u bench.py --sens /tmp/synthetic_$a.sens ${b//,/ }; summ $O/sens_$a.log ;;
    trace) run trace_$a 600 rocprofv3 --kernel-trace -d $O/trace_$a -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${b//,/ }
           f=$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0])" $O/trace_$a)
           grep '^{"metric' $O/trace_$a.log | tail -1 > $O/trace_$a.json
           python3 tools/stream_timeline.py $f $O/trace_$a.json > $O/timeline_$a.txt; python3 tools/overlap_attr.py $f $O/trace_$a.json >> $O/timeline_$a.txt
           python3 tools/trace_tail.py $f $O/trace_$a.json $O/trace_tail_$a.csv.gz
           cat $O/timeline_$a.txt; rm -rf $O/trace_$a ;;
    py) run $a $b python -u ${c//,/ } ;;
    avail) run avail 120 rocprofv3 --list-avail ;;
    kstats) run kstats_$a 600 rocprofv3 --kernel-trace --stats -d $O/kstats_$a -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${b//,/ }
            cp "$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0])" $O/kstats_$a)" $O/kstats_$a.csv
            rm -rf $O/kstats_$a; cut -d, -f1-8 $O/kstats_$a.csv | head -40 ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
