"""Every counter of the named kernels' dispatches (rocprofv3 --pmc CSV), in dispatch order.
usage: pmc_dispatch.py <dir with *counter_collection.csv> kernel [kernel ...]"""
import csv
import glob
import os
import sys

d, names = sys.argv[1], sys.argv[2:]
pc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
per = {}
for r in csv.DictReader(open(pc[0])):
    n = r["Kernel_Name"]
    if not any(x in n for x in names):
        continue
    key = (int(r["Dispatch_Id"]), n.split("(")[0].split("::")[-1])
    c = per.setdefault(key, {})
    c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for (did, n), c in sorted(per.items()):
    print(f"{n} #{did}: " + " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
