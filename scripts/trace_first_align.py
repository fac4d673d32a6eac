import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine
# C4F (env C4F=1): 4 % clutter and 40 debris blobs, bench.py's gate-rejecting config
kw = dict(clutter=0.04, debris=40_000) if os.environ.get("C4F") == "1" else {}
scan, cad, T = synth.scan_vs_cad(5_000_000, 5_000_000, **kw)
e = GICPEngine(); e.set_target_xyz(cad); e.set_source_xyz(scan); e.align(); e.close()
print("---- second context (warm process) ----", file=sys.stderr, flush=True)
e = GICPEngine()
if os.environ.get("SOURCE_FIRST") == "1":  # the reference's order (GICPAlignment.cpp:89-90)
    e.set_source_xyz(scan); e.set_target_xyz(cad)
else:
    e.set_target_xyz(cad); e.set_source_xyz(scan)
e.align(); print(e.last_result, file=sys.stderr)
e.align(); print(e.last_result, file=sys.stderr)
