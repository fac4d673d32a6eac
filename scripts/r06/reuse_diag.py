"""r06: why does a context that aligned C4 align C4F differently from a fresh one?  Compare, step by step,
a reused context with a fresh one: covariances, a first sweep at I, objective sums, then the align."""
import os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
mode = sys.argv[2] if len(sys.argv) > 2 else "c4"
scan, cad, _ = synth.scan_vs_cad(n, n, clutter=0.04, debris=n // 125)
s4, t4, _ = synth.scan_vs_cad(n, n)


def run(reuse, stage):
    e = GICPEngine(options={"target_cache": 0})
    if reuse:
        if mode == "c4":
            e.set_source_xyz(s4); e.set_target_xyz(t4)
        else:
            e.set_source_xyz(scan); e.set_target_xyz(cad)
        e.align(); e.align()
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    out = {}
    if stage == "cov":
        out["cs"] = e.debug_covariances("source", len(scan))
        out["ct"] = e.debug_covariances("target", len(cad))
    elif stage == "corr":
        out["corr"] = e.debug_correspondences(np.eye(4, dtype=np.float32), len(scan))
        out["sums"] = e.debug_fdf_sums(np.array([0.001, -0.002, 0.0005, 0.0003, -0.0002, 0.0004]))
    else:
        T = e.align()
        out["T"] = T
        out["res"] = (e.last_result["iterations"], e.last_result["n_evals"], e.last_result["n_corr"])
        out["trace"] = e.debug_trace(101)
    e.close()
    return out


for stage in ("cov", "corr", "align"):
    a, f = run(True, stage), run(False, stage)
    for k in a:
        if k == "corr":
            same = a[k][0] == f[k][0] and np.array_equal(a[k][1], f[k][1]) and np.array_equal(a[k][2], f[k][2])
            extra = f"m {a[k][0]} vs {f[k][0]}, idx diff {int((a[k][1] != f[k][1]).sum())}, M diff rows {int((a[k][2] != f[k][2]).any(axis=1).sum())}"
        elif k == "res":
            same = a[k] == f[k]
            extra = f"{a[k]} vs {f[k]}"
        elif k == "trace":
            same = len(a[k]) == len(f[k]) and all(np.array_equal(x, y) for x, y in zip(a[k], f[k]))
            extra = " ".join(f"{np.linalg.norm(np.asarray(x, np.float64) - np.asarray(y, np.float64)):.2e}" for x, y in zip(a[k], f[k]))
        else:
            A, F = np.asarray(a[k]), np.asarray(f[k])
            same = np.array_equal(A, F)
            extra = "" if same else f"rows differing {int((A != F).reshape(len(A), -1).any(axis=1).sum()) if A.ndim > 1 else int((A != F).sum())}, max {np.abs(A - F).max():.3e}"
        print(f"{mode} {stage} {k}: {'SAME' if same else 'DIFF'} {extra}", flush=True)
