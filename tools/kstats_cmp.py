"""Side-by-side average durations (us) of the named kernels in rocprofv3 --stats CSVs (kernel_stats.csv).
Usage: python tools/kstats_cmp.py A.csv [B.csv ...] [-k kernel,kernel,...]"""
import csv
import re
import sys

DEFAULT = ["k_apply_ops", "k_alloc_collect_ops", "k_compactify_ops", "k_gc", "k_alloc_insert", "k_alloc_birth",
           "k_begin_ops_tiles", "k_pcg_persist", "k_scan_keys"]


def load(path):
    out = {}
    for r in list(csv.reader(open(path)))[1:]:
        m = re.search(r"::(k_\w+)", r[0])
        if not m:
            continue
        k = m.group(1)
        calls, total = int(r[1]), float(r[2])
        c0, t0 = out.get(k, (0, 0.0))
        out[k] = (c0 + calls, t0 + total)
    return out


def main(argv):
    kernels = DEFAULT
    if "-k" in argv:
        i = argv.index("-k")
        kernels = argv[i + 1].split(",")
        argv = argv[:i] + argv[i + 2:]
    tabs = [(p, load(p)) for p in argv]
    print(f"{'kernel':22s}" + "".join(f"{p.split('/')[-1][:22]:>24s}" for p, _ in tabs))
    for k in kernels:
        row = f"{k:22s}"
        for _, t in tabs:
            c, tot = t.get(k, (0, 0.0))
            row += f"{(tot / c / 1e3 if c else float('nan')):>16.2f} ({c:6d})"
        print(row)


if __name__ == "__main__":
    main(sys.argv[1:])
