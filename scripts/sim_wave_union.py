"""CPU model of the 1-NN sweep's work at cell granularity (design study, not product code).

For sampled waves of 64 Morton-ordered queries of the C4 scene it counts the candidate points an
exact search with perfect cell pruning must test (cells whose box lies within the query's exact NN
distance): per lane (mean and max over the wave: a divergent per-lane search pays ~max) and for
the wave's union (a wave-uniform search in which every lane tests every candidate of the union).

usage: python scripts/sim_wave_union.py [n_points] [n_waves] [sweep_shift_mm]
"""
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
    nw = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
    scan, cad, T = synth.scan_vs_cad(n, n)
    q = scan.astype(np.float64)
    if len(sys.argv) > 3:  # later sweeps: queries moved towards the truth by a residual pose error
        Tinv = np.linalg.inv(T)
        frac = float(sys.argv[3])
        qt = q @ Tinv[:3, :3].T + Tinv[:3, 3]
        q = qt + frac * (q - qt)
    tgt = cad.astype(np.float64)
    lo = tgt.min(0)
    # cell size: 10 points per non-empty cell
    h = 0.005
    for _ in range(8):
        k = np.floor((tgt - lo) / h).astype(np.int64)
        key = (k[:, 2] * 4096 + k[:, 1]) * 4096 + k[:, 0]
        occ = n / len(np.unique(key))
        h *= (10.0 / occ) ** 0.5
    k = np.floor((tgt - lo) / h).astype(np.int64)
    key = (k[:, 2] * 4096 + k[:, 1]) * 4096 + k[:, 0]
    uk, cnt = np.unique(key, return_counts=True)
    cells = dict(zip(uk.tolist(), cnt.tolist()))
    print(f"h = {h * 1e3:.2f} mm, occupancy {n / len(uk):.1f}, cells {len(uk)}")
    tree = cKDTree(tgt)
    # Morton order over the query bbox, 1024 steps per axis
    qlo, qhi = q.min(0), q.max(0)
    inv = 1023.0 / (qhi - qlo).max()
    iq = np.clip(((q - qlo) * inv).astype(np.int64), 0, 1023)
    mk = spread3(iq[:, 0]) | (spread3(iq[:, 1]) << 1) | (spread3(iq[:, 2]) << 2)
    order = np.argsort(mk, kind="stable")
    rng = np.random.default_rng(0)
    waves = rng.choice(n // 64, size=nw, replace=False)
    per_mean, per_max, uni, ucells, rowsU = [], [], [], [], []
    dd = []
    sub = {}
    for w in waves:
        idx = order[w * 64:(w + 1) * 64]
        Q = q[idx]
        d, _ = tree.query(Q)
        dd.append(d)
        c = np.floor((Q - lo) / h).astype(np.int64)
        R = np.ceil(d / h).astype(np.int64) + 1
        union = set()
        per = []
        lane_cells = []
        for l in range(64):
            r = R[l]
            rr = np.arange(-r, r + 1)
            gx, gy, gz = np.meshgrid(rr + c[l, 0], rr + c[l, 1], rr + c[l, 2], indexing="ij")
            gx, gy, gz = gx.ravel(), gy.ravel(), gz.ravel()
            # gap from the query to each cell box
            def gap(g, qc, o):
                lo_ = o + g * h
                return np.maximum(np.maximum(lo_ - qc, qc - (lo_ + h)), 0.0)
            g2 = gap(gx, Q[l, 0], lo[0]) ** 2 + gap(gy, Q[l, 1], lo[1]) ** 2 + gap(gz, Q[l, 2], lo[2]) ** 2
            sel = g2 <= d[l] ** 2
            keys = ((gz[sel] * 4096 + gy[sel]) * 4096 + gx[sel]).tolist()
            tot = 0
            lane_cells.append({kk for kk in keys if cells.get(kk, 0)})
            for kk in keys:
                m = cells.get(kk, 0)
                if m:
                    tot += m
                    union.add(kk)
            per.append(tot)
        per_mean.append(np.mean(per))
        per_max.append(np.max(per))
        uni.append(sum(cells[kk] for kk in union))
        for gsz in (32, 16, 8):
            gu = []
            for g0 in range(0, 64, gsz):
                su = set().union(*lane_cells[g0:g0 + gsz])
                gu.append(sum(cells[kk] for kk in su))
            sub.setdefault(gsz, []).append(max(gu))
        ucells.append(len(union))
        rowsU.append(len({kk // 4096 for kk in union}))
    dd = np.concatenate(dd)
    print(f"NN distance mm: mean {dd.mean() * 1e3:.2f} p50 {np.median(dd) * 1e3:.2f} p90 "
          f"{np.percentile(dd, 90) * 1e3:.2f} max {dd.max() * 1e3:.2f}")
    print(f"per-lane candidates (perfect cell pruning): mean {np.mean(per_mean):.1f}, "
          f"wave max {np.mean(per_max):.1f}")
    print(f"wave union: candidates {np.mean(uni):.1f} (p90 {np.percentile(uni, 90):.0f}), "
          f"non-empty cells {np.mean(ucells):.1f}, rows {np.mean(rowsU):.1f}")
    for gsz, v in sub.items():
        print(f"groups of {gsz}: max over the wave's groups of the group-union candidates {np.mean(v):.1f}")


if __name__ == "__main__":
    main()
