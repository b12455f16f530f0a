"""The bench's timed region in a rocprofv3 trace or counter CSV: bench.py's roofline.launches k_apply_ops
dispatches that come before the end phase's last roofline.launches_after ones (the end-of-sequence
re-integration batches run the same kernel after the timed region)."""
import json


def bench_counts(bench_json):
    d = json.loads(open(bench_json).read().strip().splitlines()[-1])
    r = d["roofline"]
    return int(r["launches"]), int(r.get("launches_after", 0))


def window(seq, launches, after):
    """the timed region's items of a dispatch-ordered sequence of k_apply_ops dispatches"""
    end = len(seq) - after
    return seq[max(0, end - launches):end]


def region_bounds(rows, launches, after):
    """(t0, t1) of the timed region in a kernel trace (rows: dicts with Kernel_Name / Start_Timestamp /
    End_Timestamp): from the first timed batch's k_begin_ops_tiles to the end of the last timed k_apply_ops'
    garbage collection (the last scene kernel before the next batch)"""
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    idx = window([i for i, r in enumerate(rows) if "k_apply_ops" in r["Kernel_Name"]], launches, after)
    first, last = idx[0], idx[-1]
    while first > 0 and "k_begin_ops_tiles" not in rows[first]["Kernel_Name"]:
        first -= 1
    end = int(rows[last]["End_Timestamp"])
    for r in rows[last + 1:]:
        if "k_begin_ops_tiles" in r["Kernel_Name"] or "k_apply_ops" in r["Kernel_Name"]:
            break
        if "k_gc_" in r["Kernel_Name"]:
            end = max(end, int(r["End_Timestamp"]))
    return int(rows[first]["Start_Timestamp"]), end


def region_end_all(rows, t1, idle_ns=5_000_000):
    """end of the timed region on every stream: the last kernel end after t1 before the first idle stretch of
    idle_ns with no kernel running (bench.py synchronizes, then reads stats before its next phase)"""
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    end = t1
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t1:
            end = max(end, e) if e > t1 else end
            continue
        if s > end + idle_ns:
            break
        end = max(end, e)
    return end
