"""Scene-stream idle time in the bench's timed region, attributed to what ended it: for each gap between
scene-stream kernels (tools/trace_tail.py output), the kernel of another stream that ended last before the
scene stream resumed (the input preprocessing, a bundling kernel whose result the host waited for, or
nothing: host launch latency). Usage: gap_attr.py TRACE_TAIL.csv.gz FRAMES"""
import csv
import gzip
import re
import sys
from collections import defaultdict

SCENE = ("k_begin_ops_tiles", "k_alloc_collect_ops", "k_alloc_insert", "k_alloc_birth", "k_compactify_ops", "k_apply_ops",
         "k_gc")
INPUT = ("k_erode", "k_gauss", "k_resample", "k_depth_u16", "k_color", "k_cache_", "copyBuffer")


def name(r):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    return re.split(r"[<(]", n)[0].replace("bf::", "")


def main():
    path, frames = sys.argv[1], int(sys.argv[2])
    rows = sorted(csv.DictReader(gzip.open(path, "rt")), key=lambda r: int(r["Start_Timestamp"]))
    scene = [r for r in rows if any(k in r["Kernel_Name"] for k in SCENE)]
    other = [r for r in rows if not any(k in r["Kernel_Name"] for k in SCENE)]
    by = defaultdict(float)
    prev = None
    for r in scene:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev is not None and s > prev:
            ends = [(int(o["End_Timestamp"]), name(o)) for o in other if prev < int(o["End_Timestamp"]) <= s]
            cause = max(ends)[1] if ends else "<none: host>"
            kind = "input" if any(k in cause for k in INPUT) else ("host" if cause.startswith("<none") else "bundling")
            by[kind] += s - prev
            by["  " + cause] += s - prev
        prev = max(prev or 0, e)
    print(f"scene-stream idle per frame over {frames} frames, by what ended each gap (us):")
    for k, v in sorted(by.items(), key=lambda kv: (kv[0].startswith("  "), -kv[1])):
        if not k.startswith("  ") or v / frames / 1e3 >= 0.5:
            print(f"  {k:32s} {v / frames / 1e3:7.1f}")


if __name__ == "__main__":
    main()
