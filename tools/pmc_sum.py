"""Sums rocprofv3 --pmc counter rows per (kernel, counter) over the dispatches of k_ingest /
k_merge kernels in a pmc output directory (development)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
tot, disp = {}, {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        name = "k_ingest" if "k_ingest" in k else "k_merge" if "k_merge" in k else None
        if name is None:
            continue
        c = row["Counter_Name"]
        tot[(name, c)] = tot.get((name, c), 0.0) + float(row["Counter_Value"])
        disp.setdefault((name, c), set()).add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
for (name, c), v in sorted(tot.items()):
    n = len(disp[(name, c)])
    print("%-9s %-24s per dispatch %14.1f  (%d dispatches)" % (name, c, v / max(n, 1), n))
