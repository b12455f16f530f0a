"""Durations and gaps of consecutive k_pcg_pairs launches in a rocprofv3 kernel trace of a standalone
solve (tools/time_ba.py): where a PCG iteration's time goes. Usage: pcg_standalone.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
pcg = [k for k in K if "k_pcg_pairs" in k[2]]
dur = sorted(k[1] - k[0] for k in pcg)
gaps = sorted(b[0] - a[1] for a, b in zip(pcg, pcg[1:]) if 0 <= b[0] - a[1] < 50000)
q = lambda v, p: v[int(p * (len(v) - 1))] / 1000.0
print(f"{len(pcg)} k_pcg_pairs launches")
print("duration us: p10 %.2f p50 %.2f p90 %.2f mean %.2f" % (q(dur, .1), q(dur, .5), q(dur, .9), sum(dur) / len(dur) / 1e3))
print("gap us:      p10 %.2f p50 %.2f p90 %.2f mean %.2f" % (q(gaps, .1), q(gaps, .5), q(gaps, .9), sum(gaps) / len(gaps) / 1e3))
