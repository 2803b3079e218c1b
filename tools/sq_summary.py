"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch)."""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "?")[:60]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        # one row per dispatch (rocprofv3 already sums over dimensions)
        print(f"   {c:28s} mean/dispatch {sum(v) / len(v):.4g}  (n={len(v)})")
