"""r05: the reference's call pattern at C4 -- a fresh context, set_source, set_target, align, align
(GICPState's cycle + the unit test's iterate()) -- repeated; per align the loop time and iterations.
usage: [MGICP_LIB_NAME=...] python3 scripts/r05/cold_pair.py [reps] [C4F]"""
import os, sys, time, json
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
c4f = len(sys.argv) > 2 and sys.argv[2] == "C4F"  # the gate-rejecting workload (clutter + debris)
scan, cad, _ = synth.scan_vs_cad(5_000_000, 5_000_000, clutter=0.04 if c4f else 0.0, debris=40_000 if c4f else 0)
out = []
for r in range(reps):
    # MGICP_COLD_OPTS="name=value,...": debug options of the engines (A/B runs)
    opts = {k: float(v) for k, v in (kv.split("=") for kv in os.environ.get("MGICP_COLD_OPTS", "").split(",") if kv)}
    e = GICPEngine(options=opts)
    t0 = time.perf_counter()
    e.set_source_xyz(scan)
    t1 = time.perf_counter()
    e.set_target_xyz(cad)
    t2 = time.perf_counter()
    al = []
    for a in range(2):
        ta = time.perf_counter()
        e.align()
        tb = time.perf_counter()
        lr = e.last_result
        al.append({"wall": round(1e3 * (tb - ta), 3), "loop": round(lr["ms_loop"], 3), "prep": round(lr["ms_prep"], 3),
                   "its": lr["iterations"], "passes": lr["n_evals"]})
    e.close()
    out.append({"set_source": round(1e3 * (t1 - t0), 3), "set_target": round(1e3 * (t2 - t1), 3), "aligns": al})
    print(json.dumps(out[-1]), flush=True)
lib = os.environ.get("MGICP_LIB_NAME", "libmgicp.so")
print(lib, "first-align loop ms (median of reps 2..):", float(np.median([o["aligns"][0]["loop"] for o in out[1:]])),
      "second:", float(np.median([o["aligns"][1]["loop"] for o in out[1:]])),
      "ms-to-converge first:", float(np.median([o["set_source"] + o["set_target"] + o["aligns"][0]["wall"] for o in out[1:]])))
