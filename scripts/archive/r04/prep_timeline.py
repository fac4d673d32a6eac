#!/usr/bin/env python3
"""Timeline of the second (warm-process) context's first align from a rocprofv3 kernel trace of
scripts/trace_first_align.py: per kernel name, count / total device time inside the window from the
first kernel after the marker launch to the end of that align's loop, plus idle gaps.
usage: prep_timeline.py TRACE_DIR"""
import csv, glob, sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the marker: the second context starts after the first context's last fdf_server launch ends; take
# the window between the 2nd-to-last gap > 5 ms (process / context setup) and the start of the last align
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70]) for r in rows]
gaps = [(ev[i + 1][0] - ev[i][1], i + 1) for i in range(len(ev) - 1)]
big = [i for g, i in gaps if g > 5_000_000]
start = big[-1] if big else 0
win = ev[start:]
# stop at the second fdf_server launch group of the window's last align: take everything up to the end of the first align (3 server launches)
nsrv = 0
end = len(win)
for k, (s, e, n) in enumerate(win):
    if "fdf_server_kernel<false" in n:
        nsrv += 1
        if nsrv == 3:
            # the rest of this align: until the next correspond kernel after a gap > 1 ms
            end = k + 1
            break
win = win[:end]
t0, t1 = win[0][0], win[-1][1]
busy = defaultdict(lambda: [0, 0])
idle = 0
for k, (s, e, n) in enumerate(win):
    busy[n][0] += 1
    busy[n][1] += e - s
    if k:
        idle += max(0, s - win[k - 1][1])
print(f"window {(t1 - t0) / 1e6:.3f} ms, kernels {len(win)}, idle between kernels {idle / 1e6:.3f} ms")
for n, (c, t) in sorted(busy.items(), key=lambda x: -x[1][1])[:30]:
    print(f"  {t / 1e6:8.3f} ms  x{c:4d}  {n}")
# phases: first correspond kernel marks the end of prep
k0 = next((k for k, (s, e, n) in enumerate(win) if "correspond" in n), None)
if k0 is not None:
    print(f"prep (first kernel -> first sweep) {(win[k0][0] - t0) / 1e6:.3f} ms, loop {(t1 - win[k0][0]) / 1e6:.3f} ms")
    gl = sorted(((win[k + 1][0] - win[k][1], win[k][2], win[k + 1][2]) for k in range(k0)), reverse=True)[:12]
    for g, a, b in gl:
        print(f"   gap {g / 1e3:8.1f} us after {a} before {b}")
# r04: every kernel of the window in launch order (name, start offset, duration) -- the lazy
# covariance launches are told apart by position
print("kernels in order (start ms, duration us):")
for s, e, n in win:
    if (e - s) > 20_000:
        print(f"  {(s - t0) / 1e6:8.3f}  {(e - s) / 1e3:8.1f}  {n}")
