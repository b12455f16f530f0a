"""Average per-dispatch PMC counters of the kernels matching a regex (rocprofv3 counter csv)."""
import csv
import re
import sys
from collections import defaultdict

path, rx = sys.argv[1], re.compile(sys.argv[2])
per = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(path)):
    if rx.search(r.get("Kernel_Name", "")):
        per[r["Counter_Name"]][r.get("Dispatch_Id") or r.get("Correlation_Id")] += float(r["Counter_Value"])
for name, d in sorted(per.items()):
    print(f"{name:28s} dispatches={len(d):6d} avg={sum(d.values()) / max(1, len(d)):.4g}")
