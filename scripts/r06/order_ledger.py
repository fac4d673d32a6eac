"""r06 summation-order ledger: the oracle's full align at a config under several
summation orders of its objective passes -- the trajectory of PCL's restated BFGS is a knife-edge, so
this measures how many valid orders give the oracle's iteration count and how far T moves.

Orders: seq (input order, 1 thread: PCL's own order), omp<N> (N OpenMP parts, what the GPU parity
tests' oracle runs), rev (reversed sequential), tree:<order> (the engine's fixed chunk -> super ->
total tree, gicp_ref.c fdf_tree, over a stream order), seq:<order> (sequential over that order);
stream orders: input (source input order), morton (30-bit Morton codes over the source's own bbox,
stable in the input index), engine (the stream order the engine's grid gives, saved on the GPU box by
scripts/r06/dump_order.py, --engine-order file.npy: position -> original index).  A "+upper" suffix runs
the order with the Mahalanobis matrix's upper triangle mirrored (the engine's 6-entry storage) instead of
PCL's full Eigen inverse.
usage: python3 scripts/r06/order_ledger.py C4F [--orders seq,rev,tree:morton,...] [--out file.json]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
from leica_point_cloud_processing_amd import synth  # noqa: E402
from oracle import ref  # noqa: E402

CONFIGS = {
    "C2": dict(n=100_000, nt=100_000),
    "C2F": dict(n=100_000, nt=100_000, clutter=0.04, debris=800),
    "C4": dict(n=5_000_000, nt=5_000_000),
    "C4F": dict(n=5_000_000, nt=5_000_000, clutter=0.04, debris=40_000),
    "C5": dict(n=20_000_000, nt=5_000_000, occlusion=0.25),
}


def spread3(v):
    v = v.astype(np.uint32) & np.uint32(0x3FF)
    v = (v | (v << 16)) & np.uint32(0x030000FF)
    v = (v | (v << 8)) & np.uint32(0x0300F00F)
    v = (v | (v << 4)) & np.uint32(0x030C30C3)
    v = (v | (v << 2)) & np.uint32(0x09249249)
    return v


def morton_order(xyz):
    """the engine's morton_key_kernel over the cloud's own bbox (fp32 arithmetic), stable in input index"""
    x = np.asarray(xyz, np.float32)
    lo = x.min(axis=0)
    ext = np.float32((x.max(axis=0) - lo).max())
    inv = np.float32(1024.0) / (ext * np.float32(1.0001)) if ext > 0 else np.float32(0)
    idx = [np.clip(((x[:, d] - lo[d]) * inv).astype(np.int32), 0, 1023) for d in range(3)]
    key = spread3(idx[0]) | (spread3(idx[1]) << 1) | (spread3(idx[2]) << 2)
    return np.argsort(key, kind="stable").astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--orders", default="seq,omp8,rev,tree:input,tree:morton,seq:morton")
    ap.add_argument("--threads", type=int, default=8, help="threads for the trees / covariances / sweeps")
    ap.add_argument("--engine-order", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    c = CONFIGS[a.config]
    scan, cad, T_true = synth.scan_vs_cad(c["n"], c["nt"], occlusion=c.get("occlusion", 0.0),
                                          clutter=c.get("clutter", 0.0), debris=c.get("debris", 0))
    orders = {"input": np.arange(len(scan), dtype=np.uint32), "morton": morton_order(scan)}
    if a.engine_order:
        orders["engine"] = np.load(a.engine_order).astype(np.uint32)
    o = ref.RefGICP(threads=a.threads)
    o.set_source(scan)
    o.set_target(cad)
    rows = []
    base = None
    for name in a.orders.split(","):
        # "+upper": the Mahalanobis matrix's upper triangle mirrored (the engine's 6-entry storage)
        upper = name.endswith("+upper")
        o.set_mahalanobis_upper(upper)
        base_name = name[: -len("+upper")] if upper else name
        name_full = name
        name = base_name
        if name.startswith("omp"):
            o.set_params(threads=int(name[3:]))
            o.set_sum_order(0)
        else:
            o.set_params(threads=a.threads)
            o.set_sum_order(0)
            if name == "seq":
                o.set_sum_order(3, orders["input"])
            elif name == "rev":
                o.set_sum_order(2)
            else:
                kind, order = name.split(":")
                o.set_sum_order(1 if kind == "tree" else 3, orders[order])
        t0 = time.time()
        T, info = o.align()
        dt = time.time() - t0
        T = T.astype(np.float64)
        if base is None:
            base = T
        row = {"order": name_full, "iterations": int(info["iterations"]), "n_evals": int(info["n_evals"]),
               "n_corr_last": int(info["n_corr_last"]), "frob_vs_first": float(np.linalg.norm(T - base)),
               "err_vs_truth": float(np.abs(T @ T_true - np.eye(4)).max()), "s": round(dt, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    out = {"config": a.config, "rows": rows,
           "iterations_spread": sorted({r["iterations"] for r in rows}),
           "max_frob_vs_first": max(r["frob_vs_first"] for r in rows)}
    print(json.dumps({k: v for k, v in out.items() if k != "rows"}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
