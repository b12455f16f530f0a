"""In-loop timeline of the persistent global PCG (k_pcg_persist) from a rocprofv3 kernel trace (csv):
per launch, the delay from the previous BA-stream kernel's end to its start (queueing behind the
scene stream), its duration, and how much of [start, end] the scene stream's kernels overlapped.
Usage: python3 tools/persist_gaps.py run_kernel_trace.csv [first_pass] [passes]"""
import csv
import sys
from collections import Counter


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
    return n.split("::")[-1]


rows = list(csv.DictReader(open(sys.argv[1])))
K = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Stream_Id", r.get("Queue_Id", "?")))
           for r in rows)
ap = [k for k in K if k[2] == "k_apply_ops"]
scene = ap[-1][3]
# the window: voxel passes [first, first + count) (bench --steps 20 on the 5 000-frame stream: its timed
# frames are passes 4 800 .. 4 999; the end-of-sequence phase follows)
first = int(sys.argv[2]) if len(sys.argv) > 2 else max(0, len(ap) - 200)
count = int(sys.argv[3]) if len(sys.argv) > 3 else 200
t0, t1 = ap[first][0], ap[min(len(ap), first + count) - 1][1]
K = [k for k in K if t0 <= k[0] <= t1]
per = [k for k in K if k[2] == "k_pcg_persist"]
if not per:
    sys.exit("no k_pcg_persist in the window")
ba = per[0][3]
bak = [k for k in K if k[3] == ba]
sc = [k for k in K if k[3] == scene]
print("window ms %.1f; persist launches %d; BA stream kernels %s" % ((K[-1][1] - t0) / 1e6, len(per), Counter(k[2] for k in bak).most_common(8)))
delays, durs, ovl, prevk = [], [], [], Counter()
for i, k in enumerate(bak):
    if k[2] != "k_pcg_persist" or i == 0:
        continue
    p = bak[i - 1]
    delays.append(k[0] - p[1])
    prevk[p[2]] += 1
    durs.append(k[1] - k[0])
    o = sum(max(0, min(k[1], s[1]) - max(k[0], s[0])) for s in sc)
    ovl.append(o / max(1, k[1] - k[0]))
q = lambda v, p: sorted(v)[int(p * (len(v) - 1))]
print("delay after previous BA kernel us: p10 %.1f p50 %.1f p90 %.1f mean %.1f (previous: %s)" %
      (q(delays, .1) / 1e3, q(delays, .5) / 1e3, q(delays, .9) / 1e3, sum(delays) / len(delays) / 1e3, dict(prevk)))
print("duration us: p10 %.1f p50 %.1f p90 %.1f mean %.1f" % (q(durs, .1) / 1e3, q(durs, .5) / 1e3, q(durs, .9) / 1e3, sum(durs) / len(durs) / 1e3))
print("fraction of the launch overlapped by scene kernels: p50 %.2f mean %.2f" % (q(ovl, .5), sum(ovl) / len(ovl)))
busy = Counter()
for k in K:
    busy[k[3]] += k[1] - k[0]
print("busy ms per stream:", {s: round(v / 1e6, 2) for s, v in busy.items()}, "scene =", scene, "ba =", ba)

# the dense-term cache kernels (built per frame on the cache's stream beside the scene stream): duration
# when a scene k_apply_ops runs during them vs when none does
for name in ("k_cache_geometry", "k_cache_intensity", "k_depth_u16", "k_erode", "k_gauss", "k_resample"):
    ck = [k for k in K if k[2].startswith(name)]
    if not ck:
        continue
    with_ap, alone = [], []
    aps = [k for k in K if k[2] == "k_apply_ops"]
    for k in ck:
        o = sum(max(0, min(k[1], s[1]) - max(k[0], s[0])) for s in aps)
        (with_ap if o > 0 else alone).append(k[1] - k[0])
    m = lambda v: sum(v) / len(v) / 1e3 if v else float("nan")
    print("%s: %d launches, mean us %.1f; overlapping a k_apply_ops: %d (mean %.1f us); alone: %d (mean %.1f us)" %
          (name, len(ck), m([k[1] - k[0] for k in ck]), len(with_ap), m(with_ap), len(alone), m(alone)))

# every BA-stream kernel: the idle time before it (since the previous BA kernel ended), by kernel name
# (the waits for CU slots held by the scene stream's kernels), and its own duration
gapby, durby, cnt = Counter(), Counter(), Counter()
for p, k in zip(bak, bak[1:]):
    g = k[0] - p[1]
    if g > 200000:  # > 200 us: the stream was idle (no work queued), not waiting for slots
        continue
    gapby[k[2]] += g
    durby[k[2]] += k[1] - k[0]
    cnt[k[2]] += 1
print("BA stream, per kernel name: launches, mean wait before (us), mean duration (us)")
for n, c in cnt.most_common(14):
    print("  %-22s %6d  wait %7.1f  dur %7.1f" % (n, c, gapby[n] / c / 1e3, durby[n] / c / 1e3))
print("BA stream totals in the window: waits %.2f ms, kernels %.2f ms" % (sum(gapby.values()) / 1e6, sum(durby.values()) / 1e6))
