"""r06: steady-state align time at C4 (lists built: 5 warmup aligns, then 15 timed) for A/B of library
builds.  usage: MGICP_LIB_NAME=... python3 scripts/r06/steady_ab.py"""
import os, sys, time, json, hashlib
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

scan, cad, _ = synth.scan_vs_cad(5_000_000, 5_000_000)
e = GICPEngine(options={"target_cache": 0})
e.set_source_xyz(scan)
e.set_target_xyz(cad)
for _ in range(5):
    e.align()
walls, loops = [], []
for _ in range(15):
    t0 = time.perf_counter()
    e.align()
    walls.append(1e3 * (time.perf_counter() - t0))
    loops.append(e.last_result["ms_loop"])
T = np.asarray(e.getFinalTransformation(), dtype=np.float32)
print(json.dumps({"lib": os.environ.get("MGICP_LIB_NAME", "libmgicp.so"), "median_wall": round(float(np.median(walls)), 3),
                  "median_loop": round(float(np.median(loops)), 3), "min_wall": round(min(walls), 3),
                  "T_sha": hashlib.sha256(T.tobytes()).hexdigest()[:16]}), flush=True)
e.close()
