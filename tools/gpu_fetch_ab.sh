#!/bin/bash
# k_apply_ops FETCH_SIZE per launch (gfx950-corrected, bench's timed launches) for library variants,
# one --pmc pass each (kernel-trace only). Usage: tools/gpu_fetch_ab.sh TAG "name=lib ..." [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; V=$2; shift 2
mkdir -p $O
for v in $V; do
  name=${v%%=*}; lib=${v#*=}
  BF_HIP_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_apply_ops -d $O/pmc_$name -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $O/pmc_${name}_bench.json 2> $O/pmc_${name}_bench.err || { echo "$name pmc pass failed"; tail -20 $O/pmc_${name}_bench.err; exit 1; }
  python3 - "$O/pmc_$name/run_counter_collection.csv" "$O/pmc_${name}_bench.json" "$name" <<'PY'
import csv, json, sys
from collections import defaultdict
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
last = int(b["roofline"]["launches"])
v = defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if r.get("Counter_Name") == "FETCH_SIZE" and "k_apply_ops" in r.get("Kernel_Name", ""):
        v[int(r.get("Dispatch_Id") or r.get("Correlation_Id"))] += float(r["Counter_Value"])
f = [v[k] for k in sorted(v)][-last:]
print(sys.argv[3], "FETCH GB/launch %.3f" % (2 * 1024 * sum(f) / max(1, len(f)) / 1e9), "launches", len(f),
      "apply_us %.1f" % b["roofline"]["avg_launch_us"], "fps %.1f" % b["value"])
PY
  rm -rf $O/pmc_$name
done
