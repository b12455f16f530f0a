"""The measurement tools' timed-region selection (tools/timed_region.py and its users), on synthetic kernel
traces: bench.py's timed region is the `launches` k_apply_ops dispatches before the end phase's last
`launches_after`, and every tool that reports "the timed region" must take exactly those (round 4's tools took
the process's last dispatches, which were the end phase's)."""
import csv
import gzip
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TOOLS = os.path.join(os.path.dirname(HERE), "tools")
sys.path.insert(0, TOOLS)
from timed_region import bench_counts, region_bounds, region_end_all, window  # noqa: E402


def _trace(tmp_path, frames=30, end_phase=5):
    """30 frames (the last 20 are the timed region: applies of 1 ms from frame 10 on, 0.5 ms before), a bundling
    kernel, an idle stretch while bench.py reads its stats, then the end phase's batches (applies of 3 ms)"""
    rows, t = [], 0

    def k(name, dur, gap=10):
        nonlocal t
        t += gap
        rows.append({"Kernel_Name": name, "Queue_Id": "1", "Stream_Id": "1", "Start_Timestamp": str(t),
                     "End_Timestamp": str(t + dur), "Grid_Size": "1", "Workgroup_Size": "1"})
        t += dur

    for f in range(frames):
        k("k_begin_ops_tiles", 100_000)
        k("k_gauss", 40_000, gap=0)  # the next frame's input work, beside the batch
        for n in ("k_alloc_collect_ops", "k_compactify_ops"):
            k(n, 100_000)
        k("k_apply_ops", 1_000_000 if f >= 10 else 500_000)
        k("k_gc", 50_000)
    k("k_pcg_persist", 2_000_000)
    t += 10_000_000  # bench.py synchronizes and reads its stats
    for _ in range(end_phase):
        k("k_begin_ops_tiles", 100_000)
        k("k_apply_ops", 3_000_000)
    path = tmp_path / "trace.csv"
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps({"metric": "x", "roofline": {"launches": 20, "launches_after": end_phase}}) + "\n")
    return path, bench, rows


def test_window_takes_the_launches_before_the_end_phase():
    seq = list(range(100))
    assert window(seq, 20, 0) == list(range(80, 100))
    assert window(seq, 20, 30) == list(range(50, 70))
    assert window(seq, 200, 30) == list(range(0, 70))


def test_region_bounds_exclude_the_end_phase(tmp_path):
    path, bench, rows = _trace(tmp_path)
    launches, after = bench_counts(str(bench))
    assert (launches, after) == (20, 5)
    t0, t1 = region_bounds(rows, launches, after)
    applies = [r for r in rows if r["Kernel_Name"] == "k_apply_ops" and t0 <= int(r["Start_Timestamp"]) <= t1]
    assert len(applies) == 20
    assert all(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) == 1_000_000 for r in applies)
    # the region on every stream ends at the bundling kernel after the last batch, before the idle stretch
    t2 = region_end_all(rows, t1)
    pcg = next(r for r in rows if r["Kernel_Name"] == "k_pcg_persist")
    assert t2 == int(pcg["End_Timestamp"])


@pytest.mark.parametrize("tool", ["stream_timeline.py", "overlap_attr.py"])
def test_tools_report_the_timed_region(tmp_path, tool):
    path, bench, _ = _trace(tmp_path)
    out = subprocess.run([sys.executable, os.path.join(TOOLS, tool), str(path), str(bench)], capture_output=True,
                         text=True, check=True).stdout
    if tool == "stream_timeline.py":
        # the 20 timed frames' applies (1 ms each), not the end phase's 3 ms ones
        line = next(l for l in out.splitlines() if "k_apply_ops" in l)
        assert abs(float(line.split("busy")[1].split()[0]) - 1000.0) < 0.5, line
    else:
        line = next(l for l in out.splitlines() if l.startswith("k_gauss"))
        assert "dispatches    20" in line, line


def test_trace_tail_keeps_the_region(tmp_path):
    path, bench, _ = _trace(tmp_path)
    out = tmp_path / "tail.csv.gz"
    subprocess.run([sys.executable, os.path.join(TOOLS, "trace_tail.py"), str(path), str(bench), str(out)], check=True,
                   capture_output=True)
    kept = list(csv.DictReader(gzip.open(out, "rt")))
    names = [r["Kernel_Name"] for r in kept]
    assert names.count("k_apply_ops") == 20 and "k_pcg_persist" in names


def test_wave_log_reads_the_renders(tmp_path):
    """tools/wave_log.py: the BF_RENDER_WAVE_LOG / BF_SPLAT_TILE_LOG layout ({count, then count x {start, end,
    __smid, value}} per render, 100 MHz ticks)."""
    import numpy as np
    from wave_log import renders
    recs = []
    for r in range(2):
        n = 3 + r
        w = np.zeros((n, 4), np.uint64)
        w[:, 0] = 1000 + r * 500
        w[:, 1] = w[:, 0] + np.arange(1, n + 1) * 100  # 1, 2, 3 .. us
        w[:, 2] = (np.arange(n) % 8) << 6  # xcc in bits 6+
        w[:, 3] = 7
        recs += [np.array([n], np.uint64), w.ravel()]
    path = tmp_path / "log.bin"
    np.concatenate(recs).tofile(path)
    rs = renders(str(path))
    assert [len(x) for x in rs] == [3, 4]
    assert int(rs[1][3, 1] - rs[1][3, 0]) == 400
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "wave_log.py"), str(path)], capture_output=True, text=True,
                         check=True).stdout
    assert "2 renders in the log; render -1: 4 waves, span 4.0 us" in out, out
