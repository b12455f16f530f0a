"""The scene stream's timeline over the bench's timed region, from a rocprofv3 kernel trace: per frame, the
busy time of each scene-stream kernel and the idle gaps in front of each (where the stream waited: on the
preprocessing event, on the host, or for CU slots other streams held). Scene-stream kernels are identified by
name; the timed region comes from the bench line (tools/timed_region.py).
Usage: stream_timeline.py KERNEL_TRACE.csv BENCH.json"""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timed_region import bench_counts, region_bounds, region_end_all  # noqa: E402

SCENE = ("k_begin_ops_tiles", "k_alloc_collect_ops", "k_alloc_insert", "k_alloc_birth", "k_compactify_ops",
         "k_apply_ops", "k_gc")


def main():
    path = sys.argv[1]
    frames, after = bench_counts(sys.argv[2])
    allrows = list(csv.DictReader(open(path)))
    t0, t1 = region_bounds(allrows, frames, after)
    rows = [r for r in allrows if any(k in r["Kernel_Name"] for k in SCENE) and t0 <= int(r["Start_Timestamp"]) <= t1]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    others = defaultdict(float)  # the other streams' kernels inside the region (bundling, input), busy time
    for r in allrows:
        s = int(r["Start_Timestamp"])
        if t0 <= s <= t1 and not any(k in r["Kernel_Name"] for k in SCENE):
            others[r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")] += int(r["End_Timestamp"]) - s
    busy, gap = defaultdict(float), defaultdict(float)
    prev_end = None
    for r in rows:
        name = next(k for k in SCENE if k in r["Kernel_Name"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy[name] += e - s
        if prev_end is not None:
            gap[name] += max(0, s - prev_end)
        prev_end = max(prev_end or 0, e)
    wall = prev_end - int(rows[0]["Start_Timestamp"])
    n = frames
    print(f"scene stream over {n} frames: wall {wall / n / 1e3:.1f} us per frame, busy {sum(busy.values()) / n / 1e3:.1f}, "
          f"idle gaps {sum(gap.values()) / n / 1e3:.1f}")
    for k in SCENE:
        if busy[k] or gap[k]:
            print(f"  {k:20s} busy {busy[k] / n / 1e3:7.1f} us/frame   gap before {gap[k] / n / 1e3:6.1f} us/frame")
    t2 = region_end_all(allrows, t1)
    print(f"every stream: the region ends {(t2 - t1) / 1e3:.1f} us after the scene stream's last kernel "
          f"(whole region {(t2 - t0) / n / 1e3:.1f} us per frame)")
    print(f"other streams' kernels in the region (interval sums, us per frame; intervals include slot waits):")
    for k, v in sorted(others.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {k[:40]:40s} {v / n / 1e3:8.1f}")


if __name__ == "__main__":
    main()
