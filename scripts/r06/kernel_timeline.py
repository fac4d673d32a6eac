import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
def short(n):
    n = re.sub(r"\(.*", "", n); n = n.replace("void ", "").replace("mgicp::", "")
    return n[:38]
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 400
agg = {}
for r in rows[:lim]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = short(r["Kernel_Name"])
    print(f"{(s-t0)/1e6:9.3f} {(e-s)/1e3:9.1f}us q{r['Queue_Id']:>3} {nm}")
