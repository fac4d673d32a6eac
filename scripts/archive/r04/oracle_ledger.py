"""Oracle uncertainty ledger (CPU only, test infrastructure).

Every choice of the PCL 1.8.1 bfgs.h / gicp.hpp restatement that was made without the source text
 is flipped one at a time in the oracle (ref_params.variant bits, oracle/gicp_ref.h)
and the full align is re-run on the same synthetic workload: how far the iteration count, the
objective-pass count (the workload `value` times) and the final transform move if the restatement is
wrong on that one point.

usage: python scripts/r04/oracle_ledger.py CONFIG [threads] > profiles/r04/ledger/CONFIG.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from leica_point_cloud_processing_amd import synth  # noqa: E402
from oracle import ref  # noqa: E402

VARIANTS = {
    0: "as restated (gradient test 1e-2, cubic guard !(fpb != fpa), curvature c > a, caps 100/100, step 1, "
       "no-progress <= DBL_EPSILON)",
    1: "inner gradient test at gicp_epsilon_ = 1e-3 instead of 1e-2",
    2: "cubic interpolation whenever fpb is finite (GSL GSL_IS_REAL) instead of !(fpb != fpa)",
    4: "quadratic curvature test c > 0 (GSL) instead of c > a",
    8: "bracket / section iteration caps 20 / 20 instead of 100 / 100",
    16: "first trial step 0.1 instead of 1",
    32: "line-search no-progress test (a - alpha) fpa <= 0 instead of <= DBL_EPSILON",
}
CONFIGS = {"C2": (100_000, 100_000, {}), "C4": (5_000_000, 5_000_000, {}),
           "C4F": (5_000_000, 5_000_000, dict(clutter=0.04, debris=40_000)), "C3s": (1_000_000, 1_000_000, {})}


def main():
    name = sys.argv[1]
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else min(8, os.cpu_count() or 1)
    ns, nt, kw = CONFIGS[name]
    scan, cad, T_true = synth.scan_vs_cad(ns, nt, **kw)
    rows = []
    T0 = None
    for v, text in VARIANTS.items():
        o = ref.RefGICP(threads=threads, variant=v)
        o.set_source(scan)
        o.set_target(cad)
        t = time.perf_counter()
        T, info = o.align()
        dt = time.perf_counter() - t
        if v == 0:
            T0 = T
        rows.append({
            "variant": v, "choice": text, "converged": int(info["converged"]), "iterations": int(info["iterations"]),
            "objective_passes": int(info["n_evals"]), "n_corr_last": int(info["n_corr_last"]),
            "frob_vs_restated": float(np.linalg.norm(T.astype(np.float64) - T0.astype(np.float64))),
            "err_vs_truth": float(np.abs(T.astype(np.float64) @ T_true - np.eye(4)).max()),
            "wall_s": round(dt, 2),
        })
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"config": name, "n_source": ns, "n_target": nt, "threads": threads, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
