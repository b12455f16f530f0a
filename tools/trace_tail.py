"""Keeps the bench's timed region of a rocprofv3 kernel trace (every kernel from the first timed batch's
k_begin_ops_tiles on, all streams) as a gzipped CSV for offline timeline analysis.
Usage: trace_tail.py KERNEL_TRACE.csv BENCH.json OUT.csv.gz"""
import csv
import gzip
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timed_region import bench_counts, region_bounds, region_end_all  # noqa: E402


def main():
    path, out = sys.argv[1], sys.argv[3]
    frames, after = bench_counts(sys.argv[2])
    rows = list(csv.DictReader(open(path)))
    t0, t1 = region_bounds(rows, frames, after)
    t2 = region_end_all(rows, t1)
    rows = sorted((r for r in rows if t0 <= int(r["Start_Timestamp"]) <= t2 or (int(r["Start_Timestamp"]) < t0 < int(r["End_Timestamp"]))),
                  key=lambda r: int(r["Start_Timestamp"]))
    keep = ("Kernel_Name", "Queue_Id", "Stream_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size", "Workgroup_Size")
    with gzip.open(out, "wt") as f:
        w = csv.writer(f)
        w.writerow(keep)
        for r in rows:
            w.writerow([r.get(k, "") for k in keep])
    print(f"{len(rows)} kernels kept -> {out}")


if __name__ == "__main__":
    main()
