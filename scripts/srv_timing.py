"""Objective-pass timing of the resident pass server vs launched passes (mgicp_debug_pass_bench):
one correspondence sweep at the true transform of the C4 scene, then `reps` back-to-back passes
in each mode; the sums of both modes must be identical.  Variant libraries via MGICP_LIB_NAME."""
import json
import sys

import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
scan, cad, Ttrue = synth.scan_vs_cad(n, n)
e = GICPEngine()
e.set_source_xyz(scan)
e.set_target_xyz(cad)
T = np.linalg.inv(Ttrue).astype(np.float32)
m, _, _ = e.debug_correspondences(T, len(scan))
x = np.array([0.001, -0.002, 0.0005, 0.0003, -0.0002, 0.0004])
res = {"n": n, "m": int(m)}
for mode in (0, 1, 0, 1):
    ms, s = e.debug_pass_bench(x, reps, mode)
    res.setdefault(f"mode{mode}_us", []).append(round(1e3 * ms, 2))
    res.setdefault(f"mode{mode}_sums", s)
res["sums_equal"] = bool(np.array_equal(res.pop("mode0_sums"), res.pop("mode1_sums")))
print(json.dumps(res))
