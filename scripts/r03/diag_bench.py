"""r03 diagnostic: the resident server's timing form (debug_pass_bench mode 0) at 20k points."""
import sys
import numpy as np
sys.path.insert(0, ".")
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

scan, cad, Ttrue = synth.scan_vs_cad(20000, 20000)
T = np.linalg.inv(Ttrue).astype(np.float32)
x = np.array([0.001, -0.002, 0.0005, 0.0003, -0.0002, 0.0004])
for npasses in (1, 2, 3, 7):
    e = GICPEngine()
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    e.debug_correspondences(T, len(scan))
    try:
        ms, s = e.debug_pass_bench(x, npasses, 0)
        print("npasses", npasses, "ok", ms, s[:3], flush=True)
    except Exception as ex:
        print("npasses", npasses, "FAIL", ex, flush=True)
    ms1, s1 = e.debug_pass_bench(x, npasses, 1)
    print("   launched", ms1, s1[:3], flush=True)
    e.close()
