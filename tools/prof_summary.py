"""Print a rocprofv3 --stats kernel summary compactly."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].replace("bf::(anonymous namespace)::", "").split("(")[0]
    print(f"{name[:48]:48s} calls={r['Calls']:>6s} avg={float(r['AverageNs'])/1000:9.2f}us total={float(r['TotalDurationNs'])/1e6:8.2f}ms {float(r['Percentage']):5.1f}%")
