"""Gap analysis of the global PCG launches in a rocprofv3 kernel trace (csv): per k_pcg_pairs launch,
the idle time since the previous BA-stream kernel ended, and which other kernels were running
during those gaps. Usage: python3 tools/pcg_gaps.py run_kernel_trace.csv [first_frac]"""
import csv
import sys
from collections import Counter, defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
print("columns:", list(rows[0].keys()))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.9


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
    return n.split("::")[-1]


K = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
      r.get("Stream_Id", r.get("Queue_Id", "?")), r.get("Queue_Id", "?")) for r in rows]
K.sort()
print("stream -> queue:", sorted(Counter((k[3], k[4]) for k in K).items()))
ap = [k for k in K if k[2] == "k_apply_ops"]
t0, t1 = ap[-200][0], ap[-1][1]  # the bench's timed frames: the last 200 voxel passes
print("window us %.0f" % ((t1 - t0) / 1000.0))
K = [k for k in K if t0 <= k[0] <= t1]
print("busy us per stream:", {s: round(sum(k[1] - k[0] for k in K if k[3] == s) / 1000.0) for s in set(k[3] for k in K)})
pcg = [k for k in K if k[2] == "k_pcg_pairs"]
streams = Counter((k[3], k[4]) for k in pcg)
print("pcg launches", len(pcg), "streams/queues", streams)
sid = pcg[0][3]
ba = [k for k in K if k[3] == sid]
print("kernels on that stream:", Counter(k[2] for k in ba).most_common(12))
gaps, dur = [], []
for a, b in zip(ba, ba[1:]):
    if b[2] == "k_pcg_pairs" and a[2] == "k_pcg_pairs":
        gaps.append(b[0] - a[1])
        dur.append(b[1] - b[0])
gaps.sort(); dur.sort()
q = lambda v, p: v[int(p * (len(v) - 1))] / 1000.0
print("pcg->pcg gap us: p10 %.1f p50 %.1f p90 %.1f mean %.1f" % (q(gaps, .1), q(gaps, .5), q(gaps, .9), sum(gaps) / len(gaps) / 1000))
print("pcg dur us: p10 %.1f p50 %.1f p90 %.1f" % (q(dur, .1), q(dur, .5), q(dur, .9)))
# which other kernels overlap the pcg->pcg gaps (time-weighted)
other = [k for k in K if k[3] != sid]
ov = defaultdict(float)
j = 0
for a, b in zip(ba, ba[1:]):
    if not (b[2] == "k_pcg_pairs" and a[2] == "k_pcg_pairs"):
        continue
    g0, g1 = a[1], b[0]
    for k in other:
        if k[0] < g1 and k[1] > g0:
            ov[k[2]] += (min(g1, k[1]) - max(g0, k[0])) / 1000.0
tot = sum(gaps) / 1000.0
print("gap total us %.0f; overlapped by:" % tot)
for n, v in sorted(ov.items(), key=lambda x: -x[1])[:10]:
    print("  %-30s %.0f us (%.0f%%)" % (n, v, 100 * v / tot))
