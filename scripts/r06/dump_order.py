"""r06: save the engine's source stream order at a config (for the oracle's summation-order ledger)."""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd.engine import GICPEngine
sys.path.insert(0, os.path.join(os.getcwd(), "scripts", "r06"))
from order_ledger import CONFIGS  # noqa: E402
from leica_point_cloud_processing_amd import synth  # noqa: E402

name, out = sys.argv[1], sys.argv[2]
c = CONFIGS[name]
scan, cad, _ = synth.scan_vs_cad(c["n"], c["nt"], occlusion=c.get("occlusion", 0.0), clutter=c.get("clutter", 0.0),
                                 debris=c.get("debris", 0))
e = GICPEngine()
e.set_source_xyz(scan)
e.set_target_xyz(cad)
order = e.debug_source_order(len(scan))
T = e.align()
np.save(out, order)
print(name, "order saved", len(order), "iterations", e.last_result["iterations"], "n_corr", e.last_result["n_corr"])
e.close()
