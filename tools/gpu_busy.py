"""GPU busy fraction in a window of a rocprofv3 kernel trace (csv): the union of all kernels' [start, end]
intervals over the window between voxel passes [first, first + count), and each stream's busy time.
Usage: python3 tools/gpu_busy.py run_kernel_trace.csv [first_pass] [passes]"""
import csv
import sys
from collections import Counter


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
    return n.split("::")[-1]


rows = list(csv.DictReader(open(sys.argv[1])))
K = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Stream_Id", "?")) for r in rows)
ap = [k for k in K if k[2] == "k_apply_ops"]
first = int(sys.argv[2]) if len(sys.argv) > 2 else max(0, len(ap) - 200)
count = int(sys.argv[3]) if len(sys.argv) > 3 else 200
t0, t1 = ap[first][0], ap[min(len(ap), first + count) - 1][1]
W = [k for k in K if k[1] > t0 and k[0] < t1]
busy, cur_s, cur_e = 0, None, None
for s, e, *_ in W:
    s, e = max(s, t0), min(e, t1)
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
span = t1 - t0
print("window %.2f ms, %d passes; GPU busy (any kernel) %.2f ms = %.0f %%" % (span / 1e6, count, busy / 1e6, 100.0 * busy / span))
per = Counter()
for s, e, n, st in W:
    per[st] += min(e, t1) - max(s, t0)
print("per stream busy ms:", {k: round(v / 1e6, 2) for k, v in per.items()})
byk = Counter()
for s, e, n, st in W:
    byk[n] += min(e, t1) - max(s, t0)
print("top kernels (ms):", [(n, round(v / 1e6, 2)) for n, v in byk.most_common(12)])
