"""Per-dispatch durations (kernel trace) and SQ counters (PMC) of the named kernels, in launch order."""
import csv
import glob
import os
import sys

d = sys.argv[1]
names = sys.argv[2:]


def short(n):
    return n.split("(")[0].split("::")[-1]


kt = glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True)
if kt:
    rows = sorted(csv.DictReader(open(kt[0])), key=lambda r: int(r["Start_Timestamp"]))
    for n in names:
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if n in r["Kernel_Name"]]
        print(f"{n} durations us: {[round(x, 1) for x in dur]}")
pc = glob.glob(os.path.join(d, "sq", "**", "*counter_collection.csv"), recursive=True)
if pc:
    per = {}
    for r in csv.DictReader(open(pc[0])):
        n = r["Kernel_Name"]
        if not any(x in n for x in names):
            continue
        key = (short(n), int(r["Dispatch_Id"]))
        per.setdefault(key, {})[r["Counter_Name"]] = per.get(key, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for (n, did), c in sorted(per.items(), key=lambda kv: kv[0][1]):
        w = c.get("SQ_WAVES", 1) or 1
        print(f"{n} #{did}: VALU/wave {c.get('SQ_INSTS_VALU', 0) / w:.0f} SALU/wave {c.get('SQ_INSTS_SALU', 0) / w:.0f} "
              f"VMEM/wave {c.get('SQ_INSTS_VMEM', 0) / w:.1f} wait/wave-cycles {c.get('SQ_WAIT_ANY', 0) / max(c.get('SQ_WAVE_CYCLES', 1), 1):.2f} "
              f"busy {c.get('SQ_BUSY_CYCLES', 0):.3g} wave-cycles {c.get('SQ_WAVE_CYCLES', 0):.3g} active-inst {c.get('SQ_ACTIVE_INST_ANY', 0):.3g}")
