"""Design study (not product code): candidates a wave-uniform 1-NN scan tests per wave when all 64
lanes (Morton-ordered queries) iterate the same grid rows of their union box, vs the per-lane search.
  A: each needed row scanned over the union box's x-range
  B: each needed row scanned over the union of the needing lanes' x-ranges (per-row wave min / max)
Per-lane bound = exact NN distance (what the seeds approach).  usage: sim_union_rows.py [n] [waves] [frac]"""
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from leica_point_cloud_processing_amd import synth  # noqa: E402


def spread3(v):
    v = v.astype(np.uint64) & 0x3FF
    v = (v | (v << 16)) & 0x030000FF
    v = (v | (v << 8)) & 0x0300F00F
    v = (v | (v << 4)) & 0x030C30C3
    v = (v | (v << 2)) & 0x09249249
    return v


n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
nw = int(sys.argv[2]) if len(sys.argv) > 2 else 300
scan, cad, T = synth.scan_vs_cad(n, n)
q = scan.astype(np.float64)
if len(sys.argv) > 3:
    Tinv = np.linalg.inv(T)
    frac = float(sys.argv[3])
    qt = q @ Tinv[:3, :3].T + Tinv[:3, 3]
    q = qt + frac * (q - qt)
tgt = cad.astype(np.float64)
lo = tgt.min(0)
h = 0.00603
k = np.floor((tgt - lo) / h).astype(np.int64)
dims = k.max(0) + 1
lin = (k[:, 2] * dims[1] + k[:, 1]) * dims[0] + k[:, 0]
counts = np.bincount(lin, minlength=int(np.prod(dims)))
cs = np.concatenate([[0], np.cumsum(counts)])  # cell_start
tree = cKDTree(tgt)
qlo = q.min(0)
inv = 1023.0 / (q.max(0) - qlo).max()
iq = np.clip(((q - qlo) * inv).astype(np.int64), 0, 1023)
order = np.argsort(spread3(iq[:, 0]) | (spread3(iq[:, 1]) << 1) | (spread3(iq[:, 2]) << 2), kind="stable")
rng = np.random.default_rng(0)
A, B, P, rowsN, boxrows = [], [], [], [], []
for w in rng.choice(n // 64, size=nw, replace=False):
    Q = q[order[w * 64:(w + 1) * 64]]
    d, _ = tree.query(Q)
    R = d * 1.00001 + 1e-6
    c0 = np.floor((Q - R[:, None] - lo) / h).astype(np.int64)
    c1 = np.floor((Q + R[:, None] - lo) / h).astype(np.int64)
    c0 = np.maximum(c0, 0)
    c1 = np.minimum(c1, dims - 1)
    X0, Y0, Z0 = c0.min(0)
    X1, Y1, Z1 = c1.max(0)
    a = b = p = nr = 0
    boxrows.append((Y1 - Y0 + 1) * (Z1 - Z0 + 1))
    for z in range(Z0, Z1 + 1):
        gz = np.maximum(np.maximum(lo[2] + z * h - Q[:, 2], Q[:, 2] - (lo[2] + (z + 1) * h)), 0)
        for y in range(Y0, Y1 + 1):
            gy = np.maximum(np.maximum(lo[1] + y * h - Q[:, 1], Q[:, 1] - (lo[1] + (y + 1) * h)), 0)
            gyz = gy * gy + gz * gz
            need = gyz <= R * R
            if not need.any():
                continue
            nr += 1
            row = (z * dims[1] + y) * dims[0]
            a += cs[row + X1 + 1] - cs[row + X0]
            rx = np.sqrt(np.maximum(R[need] ** 2 - gyz[need], 0))
            xa = np.maximum(np.floor((Q[need, 0] - rx - lo[0]) / h).astype(np.int64), 0)
            xb = np.minimum(np.floor((Q[need, 0] + rx - lo[0]) / h).astype(np.int64), dims[0] - 1)
            b += cs[row + xb.max() + 1] - cs[row + xa.min()]
            p = max(p, 0)
    A.append(a)
    B.append(b)
    rowsN.append(nr)
print(f"frac {sys.argv[3] if len(sys.argv) > 3 else 1}: union-box rows {np.mean(boxrows):.1f}, needed rows {np.mean(rowsN):.1f}; "
      f"candidates per wave A (box x-range) {np.mean(A):.0f} (p90 {np.percentile(A, 90):.0f}), "
      f"B (per-row union x-range) {np.mean(B):.0f} (p90 {np.percentile(B, 90):.0f})")
