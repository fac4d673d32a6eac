"""r05: k-NN covariance time per 5M cloud against the grid's occupancy target (debug option grid_occ),
profiling mode on the synchronous path (as knn_time.py).
usage: python3 scripts/r05/knn_occ.py 5 7 10 14"""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

scan, cad, T = synth.scan_vs_cad(5_000_000, 5_000_000)
for occ in [float(a) for a in sys.argv[1:]]:
    e = GICPEngine(options={"target_cache": 0})
    e.set_profiling(True)
    e.set_source_xyz(scan)
    res = []
    for rep in range(4):
        e.debug_option("grid_occ", occ)
        e.set_target_xyz(cad if rep % 2 == 0 else np.ascontiguousarray(cad[::-1]))
        e.set_profiling(True)
        C = e.debug_covariances("target", len(cad))
        kt = e.kernel_times()["knn_cov"]
        res.append(kt["avg_ms"] * kt["count"])
    print(f"occ {occ}: knn_cov per 5M cloud (ms) {[round(r, 3) for r in res]} min {min(res[1:]):.3f}", flush=True)
    e.close()
