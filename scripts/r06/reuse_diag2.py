"""r06: reused vs fresh context source covariances against the oracle, under debug options."""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine
from oracle import ref

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
scan, cad, _ = synth.scan_vs_cad(n, n, clutter=0.04, debris=n // 125)
s4, t4, _ = synth.scan_vs_cad(n, n)
cs_ref = ref.covariances(scan, threads=16)


def run(reuse, opts, order):
    e = GICPEngine(options={"target_cache": 0, **opts})
    if reuse:
        e.set_source_xyz(s4); e.set_target_xyz(t4)
        e.align(); e.align()
    if order == "st":
        e.set_source_xyz(scan); e.set_target_xyz(cad)
    else:
        e.set_target_xyz(cad); e.set_source_xyz(scan)
    cs = e.debug_covariances("source", len(scan))
    e.close()
    return cs


for opts in ({}, {"lazy_src_cov": 0}, {"async_cov": 0}):
    for order in ("st", "ts"):
        for reuse in (False, True):
            cs = run(reuse, opts, order)
            bad = (cs != cs_ref).any(axis=1)
            zero = (cs == 0).all(axis=1)
            print(f"opts {opts} order {order} reuse {reuse}: rows != oracle {int(bad.sum())}, all-zero rows {int(zero.sum())}, "
                  f"max {np.abs(cs - cs_ref).max():.3e}", flush=True)
