#!/bin/bash
# gpurun with retries ONLY when the box never ran the command (status "transient", rc null): an
# infrastructure event, nothing of ours ran. Any other outcome (ok, fail, fault, timeout) returns.
# Usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6; do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  st=$(python3 -c "import json; d=json.load(open('/root/repo/gpurun_out/.last_call.json')); print(d.get('status'), d.get('rc'))" 2>/dev/null)
  case "$st" in
    "transient None") echo "[retry $i after transient infra failure]"; sleep 90 ;;
    *) exit $rc ;;
  esac
done
exit $rc
