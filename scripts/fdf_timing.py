"""Objective-pass kernel timing at C4 (5M <-> 5M) outside the BFGS loop: one correspondence sweep
at the true transform, then `reps` objective passes with per-launch HIP events
(MGICP_PROF_STRIDE=1).  Diagnostics knobs (MGICP_FDF_DIAG, MGICP_FDF_BLOCKS) come from the env."""
import json
import sys

import numpy as np

from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
scan, cad, Ttrue = synth.scan_vs_cad(n, n)
e = GICPEngine()
e.set_source_xyz(scan)
e.set_target_xyz(cad)
T = np.linalg.inv(Ttrue).astype(np.float32)
m, _, _ = e.debug_correspondences(T, len(scan))
x = np.array([0.001, -0.002, 0.0005, 0.0003, -0.0002, 0.0004])
for _ in range(5):
    e.debug_fdf_sums(x)
e.set_profiling(True)
for _ in range(reps):
    e.debug_fdf_sums(x)
kt = e.kernel_times()
print(json.dumps({"n": n, "m": int(m), "fdf_us": round(1e3 * kt["fdf"]["avg_ms"], 2), "count": kt["fdf"]["count"]}))
