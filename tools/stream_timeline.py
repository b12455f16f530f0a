"""The scene stream's timeline over the bench's timed region, from a rocprofv3 kernel trace: per frame, the
busy time of each scene-stream kernel and the idle gaps in front of each (where the stream waited: on the
preprocessing event, on the host, or for CU slots other streams held). Scene-stream kernels are identified by
name. Usage: stream_timeline.py KERNEL_TRACE.csv FRAMES"""
import csv
import sys
from collections import defaultdict

SCENE = ("k_begin_ops_tiles", "k_alloc_collect_ops", "k_alloc_insert", "k_alloc_birth", "k_compactify_ops",
         "k_apply_ops", "k_gc_identify", "k_gc_free_simple", "k_gc_free_list", "k_gc_zero")


def main():
    path, frames = sys.argv[1], int(sys.argv[2])
    rows = [r for r in csv.DictReader(open(path)) if any(k in r["Kernel_Name"] for k in SCENE)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the timed region: the last `frames` k_apply_ops dispatches and everything after the first of them
    applies = [i for i, r in enumerate(rows) if "k_apply_ops" in r["Kernel_Name"]]
    first = applies[-frames]
    # start at the scene kernels of that frame's batch (its k_begin_ops_tiles)
    while first > 0 and "k_begin_ops_tiles" not in rows[first]["Kernel_Name"]:
        first -= 1
    rows = rows[first:]
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


if __name__ == "__main__":
    main()
