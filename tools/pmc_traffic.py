"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE counts 64 B per 128-B request
on wide streaming reads, so it is doubled; WRITE_SIZE is taken as is. Both counters are in KB.
Optionally a third pass (SQ_INSTS_VALU, wave-level VALU instructions) gives the issue count per launch.
With --bench JSON (the bench line the profiled command printed), only the last
roofline.launches dispatches (bench.py's timed region) are averaged and the bench's
config.workload is recorded, so bench.py uses the figures only for that same workload.
With the bench JSON, the timed region is roofline.launches dispatches before the end phase's
roofline.launches_after (tools/timed_region.py).
Usage: pmc_traffic.py FETCH.csv WRITE.csv KERNEL_REGEX OUT.json [VALU.csv] [--bench BENCH.json]"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timed_region import window  # noqa: E402
from collections import defaultdict


def per_dispatch(path, counter, rx):
    vals = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter or not rx.search(r.get("Kernel_Name", "")):
            continue
        vals[int(r.get("Dispatch_Id") or r.get("Correlation_Id"))] += float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    argv = sys.argv[1:]
    bench = None
    if "--bench" in argv:
        i = argv.index("--bench")
        bench = json.loads(open(argv[i + 1]).read().strip().splitlines()[-1])
        del argv[i:i + 2]
    fetch_csv, write_csv, kernel, out = argv[:4]
    rx = re.compile(kernel)
    last = int(bench["roofline"]["launches"]) if bench else 0
    after = int(bench["roofline"].get("launches_after", 0)) if bench else 0
    f = per_dispatch(fetch_csv, "FETCH_SIZE", rx)
    w = per_dispatch(write_csv, "WRITE_SIZE", rx)
    if last:
        f, w = window(f, last, after), window(w, last, after)
    fetch_b = 2.0 * 1024.0 * sum(f) / max(1, len(f))
    write_b = 1024.0 * sum(w) / max(1, len(w))
    res = {"kernel": kernel, "dispatches_fetch": len(f), "dispatches_write": len(w),
           "fetch_bytes_per_launch_corrected": fetch_b, "write_bytes_per_launch": write_b,
           "bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950 half-count on 128-B requests), KB -> bytes"}
    if bench:
        res["workload"] = bench["config"]["workload"]
        res["pass_rev"] = bench["roofline"].get("pass_rev")
        res["averaged_over"] = f"{last} dispatches before the end phase's last {after} (the bench's timed region)"
        # per-unit rates (bench.py scales them by its own run's counts): fetched bytes per voxel-op
        # evaluation (the gathers and the voxel reads both grow with it), written bytes per voxel
        # read + written, VALU wave-instructions per evaluation
        pl = bench["roofline"]["per_launch"]
        res["units_per_launch"] = {"voxel_op_evaluations": pl["voxel_op_evaluations"], "voxels_rmw": pl["voxels_rmw"],
                                   "halves_loaded": pl.get("halves_loaded"),
                                   "work_list_blocks": pl["work_list_blocks"], "ops": pl["ops"]}
        res["fetch_bytes_per_evaluation"] = fetch_b / max(1.0, pl["voxel_op_evaluations"])
        res["write_bytes_per_voxel_rmw"] = write_b / max(1.0, pl["voxels_rmw"])
    if len(argv) > 4:
        v = per_dispatch(argv[4], "SQ_INSTS_VALU", rx)
        if last:
            v = window(v, last, after)
        res["dispatches_valu"] = len(v)
        res["valu_insts_per_launch"] = sum(v) / max(1, len(v))
        if bench:
            res["valu_insts_per_evaluation"] = res["valu_insts_per_launch"] / max(1.0, bench["roofline"]["per_launch"]["voxel_op_evaluations"])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
