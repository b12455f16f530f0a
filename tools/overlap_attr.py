"""Attribute in-loop kernel intervals to co-scheduling: for each kernel of interest, over the dispatches
of the bench's timed region (the last `frames` of them), the mean trace interval, the mean part of it
that overlaps a k_apply_ops dispatch, and the remainder. A kernel whose interval is mostly covered by
the voxel pass is waiting for CU slots the pass holds (its own work is its standalone time).
The timed region comes from the bench line (tools/timed_region.py).
Usage: overlap_attr.py KERNEL_TRACE.csv BENCH.json [kernel substrings...]"""
import bisect
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timed_region import bench_counts, region_bounds  # noqa: E402


def main():
    path = sys.argv[1]
    frames, after = bench_counts(sys.argv[2])
    names = sys.argv[3:] or ["k_cache_geometry", "k_cache_intensity", "k_gauss", "k_erode"]
    rows = list(csv.DictReader(open(path)))
    t0, t1 = region_bounds(rows, frames, after)
    iv = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))  # noqa: E731
    apply = sorted(iv(r) for r in rows if "k_apply_ops" in r["Kernel_Name"])
    starts = [a for a, _ in apply]

    def covered(s, e):
        # apply dispatches are serial on one stream: they do not overlap each other
        i = max(0, bisect.bisect_right(starts, s) - 1)
        c = 0
        while i < len(apply) and apply[i][0] < e:
            a, b = apply[i]
            c += max(0, min(b, e) - max(a, s))
            i += 1
        return c

    for n in names:
        d = sorted((iv(r) for r in rows if n in r["Kernel_Name"]), key=lambda x: x[0])
        d = [x for x in d if t0 <= x[0] <= t1]
        if not d:
            print(f"{n}: no dispatches")
            continue
        tot = sum(e - s for s, e in d) / len(d) / 1e3
        cov = sum(covered(s, e) for s, e in d) / len(d) / 1e3
        print(f"{n:20s} dispatches {len(d):5d}  interval {tot:8.1f} us  overlapped by k_apply_ops {cov:8.1f} us "
              f"({100 * cov / max(tot, 1e-9):5.1f} %)  rest {tot - cov:7.1f} us")


if __name__ == "__main__":
    main()
