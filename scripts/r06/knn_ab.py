"""r06: k-NN covariance time per 5M cloud with the fp64 finish inside the search (knn_split 0) and in
knn_finish_kernel (knn_split 1), alternating; profiling mode (HIP events around the k-NN family: search,
finish and hand-off launches) on the synchronous path, a fresh target each repeat.
usage: python3 scripts/r06/knn_ab.py [reps]"""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
scan, cad, T = synth.scan_vs_cad(5_000_000, 5_000_000)
out = {0: [], 1: []}
ref = None
for rep in range(reps):
    for split in (0, 1):
        e = GICPEngine(options={"knn_split": split, "async_cov": 0})
        e.set_source_xyz(scan[:1000])
        e.set_target_xyz(cad if rep % 2 == 0 else np.ascontiguousarray(cad[::-1]))
        e.set_profiling(True)
        c = e.debug_covariances("target", len(cad))
        kt = e.kernel_times()["knn_cov"]
        out[split].append(kt["avg_ms"] * kt["count"])
        if rep % 2 == 0:
            if ref is None:
                ref = c
            assert np.array_equal(c, ref), "split changed the covariances"
        e.close()
for s in (0, 1):
    print(f"knn_split {s}: ms per 5M cloud {[round(v, 3) for v in out[s]]} median {np.median(out[s][1:]):.3f}")
