"""Summarise rocprofv3 --pmc counter CSVs under a directory: per kernel, mean per dispatch."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k)
    for c, v in sorted(cs.items()):
        # several dispatches per pass: values are per dispatch (summed over XCD instances)
        print(f"  {c:24s} {sum(v) / max(1, len(set(range(len(v))))):16.1f}  (n={len(v)})")
