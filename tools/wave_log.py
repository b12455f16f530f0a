"""Summarise a BF_RENDER_WAVE_LOG file (raycast.hip): per render, when the renderKernel's waves start and end
relative to the first wave's start, how long they run, how many run at once, and the spread over XCDs.
Clock: s_memrealtime, 100 MHz (10 ns ticks).  Usage: python tools/wave_log.py LOG [RENDER_INDEX (default -1)]"""
import sys

import numpy as np


def renders(path):
    raw = np.fromfile(path, dtype=np.uint64)
    i, out = 0, []
    while i < raw.size:
        n = int(raw[i])
        out.append(raw[i + 1:i + 1 + 4 * n].reshape(n, 4))
        i += 1 + 4 * n
    return out


def main():
    rs = renders(sys.argv[1])
    k = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    w = rs[k].astype(np.int64)
    w = w[w[:, 1] > 0]  # waves that ran (the log is sized for either tile shape)
    t0 = w[:, 0].min()
    start, end = (w[:, 0] - t0) * 10e-3, (w[:, 1] - t0) * 10e-3  # microseconds
    dur = end - start
    pc = lambda a: " ".join(f"p{q} {np.percentile(a, q):7.1f}" for q in (0, 10, 50, 90, 100))
    print(f"{len(rs)} renders in the log; render {k}: {len(w)} waves, span {end.max():.1f} us")
    print("start us   ", pc(start))
    print("duration us", pc(dur))
    print("end us     ", pc(end))
    print("longest per-lane march: mean %.1f max %d" % (w[:, 3].mean(), w[:, 3].max()))
    # concurrency over time (waves resident)
    ts = np.linspace(0, end.max(), 21)
    conc = [int(((start <= t) & (end > t)).sum()) for t in ts]
    print("resident waves at 0..100 % of the span:", conc)
    xcc = w[:, 2] >> 6  # __smid on gfx950: xcc << 6 | se << 4 | cu
    for x in np.unique(xcc):
        m = xcc == x
        print(f"  xcc {x}: waves {m.sum():5d}  mean duration {dur[m].mean():7.1f} us  last end {end[m].max():7.1f} us")
    # duration against the wave's march length
    for lo, hi in ((0, 6), (6, 10), (10, 14), (14, 100)):
        m = (w[:, 3] >= lo) & (w[:, 3] < hi)
        if m.any():
            print(f"  march {lo:2d}-{hi:3d} samples: {m.sum():5d} waves, mean duration {dur[m].mean():7.1f} us")


if __name__ == "__main__":
    main()
