#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc CSVs under a directory.
usage: pmc_kernels.py DIR [KERNEL_SUBSTR ...]"""
import csv, glob, os, sys
from collections import defaultdict

d = sys.argv[1]
subs = sys.argv[2:]
acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name", "")
            if subs and not any(s in k for s in subs):
                continue
            acc[k.split("(")[0][-40:]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} avg {sum(v)/len(v):16.1f}  n={len(v)}")
