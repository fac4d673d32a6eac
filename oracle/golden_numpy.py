"""TEST INFRASTRUCTURE ONLY: an independent NumPy/SciPy restatement of PCL 1.8.1 GICP and the
generator of the committed golden fixtures under tests/golden/.

The reference (catec/leica_point_cloud_processing) delegates the whole hot path to PCL 1.8.1
(include/GICPAlignment.h:153), which is neither vendored under /root/reference nor installed
here, so the reference itself cannot be run (DESIGN.md "Oracle").  The C oracle
(oracle/gicp_ref.c) is therefore pinned two ways:
  1. the reference's own known-answer scenario: test/test_gicp_alignment.cpp samples
     test/cube.ply (5000 points, glibc rand()) and rotates it by yaw 0.175 rad, so GICP must
     return Rz(0.175) -- the fixture input is regenerated bit-exactly (synth.cube_fixture);
  2. this second, independently written restatement (scipy cKDTree k-NN, numpy eigh, batched
     numpy inverse, a Python port of bfgs.h), whose outputs are frozen as fixtures.

Run:  python -m oracle.golden_numpy      (writes tests/golden/*.npz)
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

f32 = np.float32


# ---------------------------------------------------------------------------------------
def knn_exact(pts: np.ndarray, queries: np.ndarray, k: int):
    """k nearest by (float32 d^2, index): scipy candidates re-ranked with float32 distances."""
    tree = cKDTree(pts.astype(np.float64))
    kk = min(len(pts), k + 8)
    _, idx = tree.query(queries.astype(np.float64), k=kk)
    idx = idx.reshape(len(queries), kk)
    d = queries[:, None, :].astype(np.float32) - pts[idx].astype(np.float32)
    d2 = d[..., 0] * d[..., 0]
    d2 = d2 + d[..., 1] * d[..., 1]
    d2 = d2 + d[..., 2] * d[..., 2]
    order = np.lexsort((idx, d2), axis=1)
    idx = np.take_along_axis(idx, order, 1)[:, :k]
    d2 = np.take_along_axis(d2, order, 1)[:, :k]
    return idx, d2


def covariances(pts: np.ndarray, k: int = 20, eps: float = 1e-3) -> np.ndarray:
    """GICP::computeCovariances; returns (n, 6) {c00,c01,c02,c11,c12,c22}."""
    pts = pts.astype(np.float32)
    nn, _ = knn_exact(pts, pts, k)
    P = pts[nn]  # (n, k, 3) float32
    mean = P.astype(np.float64).sum(1) / k
    prod = (P[:, :, :, None] * P[:, :, None, :]).astype(np.float64)  # fp32 products, then fp64
    S = prod.sum(1) / k - mean[:, :, None] * mean[:, None, :]
    w, V = np.linalg.eigh(S)
    kmin = np.argmin(np.abs(w), axis=1)
    n = V[np.arange(len(pts)), :, kmin]
    C = np.eye(3)[None] - (1.0 - eps) * n[:, :, None] * n[:, None, :]
    return np.stack([C[:, 0, 0], C[:, 0, 1], C[:, 0, 2], C[:, 1, 1], C[:, 1, 2], C[:, 2, 2]], 1)


def full3(c6):
    c = np.asarray(c6)
    return np.stack([np.stack([c[:, 0], c[:, 1], c[:, 2]], 1),
                     np.stack([c[:, 1], c[:, 3], c[:, 4]], 1),
                     np.stack([c[:, 2], c[:, 4], c[:, 5]], 1)], 1)


def xform32(T: np.ndarray, X: np.ndarray) -> np.ndarray:
    T = T.astype(np.float32)
    out = np.empty_like(X, dtype=np.float32)
    for r in range(3):
        a = T[r, 0] * X[:, 0]
        a = a + T[r, 1] * X[:, 1]
        a = a + T[r, 2] * X[:, 2]
        out[:, r] = a + T[r, 3]
    return out


# ---------------------------------------------------------------------------------------
# applyState: Eigen AngleAxisf(z)*AngleAxisf(y)*AngleAxisf(x) through quaternions, float32
def apply_state(x) -> np.ndarray:
    from leica_point_cloud_processing_amd.synth import _quat_axis, _quat_matrix, _quat_mul

    q = _quat_mul(_quat_mul(_quat_axis(float(f32(x[5])), 2), _quat_axis(float(f32(x[4])), 1)),
                  _quat_axis(float(f32(x[3])), 0))
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = _quat_matrix(q)
    T[0, 3], T[1, 3], T[2, 3] = f32(x[0]), f32(x[1]), f32(x[2])
    return T


def r_derivative(x, R):
    phi, theta, psi = x[3], x[4], x[5]
    cf, sf, ct, st, cp, sp = math.cos(phi), math.sin(phi), math.cos(theta), math.sin(theta), math.cos(psi), math.sin(psi)
    dphi = np.array([[0, sf * sp + cf * cp * st, cf * sp - cp * sf * st],
                     [0, -cp * sf + cf * sp * st, -cf * cp - sf * sp * st],
                     [0, cf * ct, -ct * sf]])
    dtheta = np.array([[-cp * st, cp * ct * sf, cf * cp * ct],
                       [-sp * st, ct * sf * sp, cf * ct * sp],
                       [-ct, -sf * st, -cf * st]])
    dpsi = np.array([[-ct * sp, -cf * cp - sf * sp * st, cp * sf - cf * sp * st],
                     [cp * ct, -cf * sp + cp * sf * st, sf * sp + cf * cp * st],
                     [0, 0, 0]])
    return [float(np.trace(d @ R)) for d in (dphi, dtheta, dpsi)]


class Functor:
    def __init__(self, S, Q, M):
        self.S, self.Q, self.M = S, Q, M
        self.m = len(S)
        self.calls = 0

    def fdf(self, x):
        self.calls += 1
        A = apply_state(x)
        pp = xform32(A, self.S)
        res = (pp - self.Q).astype(np.float64)
        t = np.einsum("nab,nb->na", self.M, res)
        f = float(np.sum(np.einsum("na,na->n", res, t))) / self.m
        g = np.zeros(6)
        g[:3] = t.sum(0) * (2.0 / self.m)
        R = self.S.astype(np.float64).T @ t * (2.0 / self.m)
        g[3:] = r_derivative(x, R)
        return f, g


# ---------------------------------------------------------------------------------------
# bfgs.h (GSL vector_bfgs2 port), written independently of oracle/gicp_ref.c
class BFGS:
    def __init__(self, fn):
        self.fn = fn
        self.rho = self.sigma = 0.01
        self.tau1, self.tau2, self.tau3 = 9.0, 0.05, 0.5
        self.order = 3
        self.step_size = 1.0
        self.iters = 100

    def _f(self, a):
        if a == self.fkey:
            return self.fa
        self.xa = self.x0 + a * self.p
        self.fa, _ = self.fn.fdf(self.xa)
        self.fkey = a
        return self.fa

    def _df(self, a):
        if a == self.dfkey:
            return self.dfa
        self.xa = self.x0 + a * self.p
        if a != self.gkey:
            _, self.ga = self.fn.fdf(self.xa)
            self.gkey = a
        self.dfa = float(self.ga @ self.p)
        self.dfkey = a
        return self.dfa

    def _fdf(self, a):
        if a == self.fkey and a == self.dfkey:
            return self.fa, self.dfa
        if a == self.fkey or a == self.dfkey:
            return self._f(a), self._df(a)
        self.xa = self.x0 + a * self.p
        self.fa, self.ga = self.fn.fdf(self.xa)
        self.fkey = self.gkey = self.dfkey = a
        self.dfa = float(self.ga @ self.p)
        return self.fa, self.dfa

    def init(self, x):
        self.delta_f = 0.0
        self.f, self.g = self.fn.fdf(x)
        self.x0, self.g0 = x.copy(), self.g.copy()
        self.g0norm = float(np.linalg.norm(self.g0))
        self.p = self.g * -1 / self.g0norm
        self.pnorm = float(np.linalg.norm(self.p))
        self.fp0 = -self.g0norm
        self.xa, self.fa, self.ga = self.x0.copy(), self.f, self.g0.copy()
        self.fkey = self.gkey = self.dfkey = 0.0
        self.dfa = float(self.ga @ self.p)

    @staticmethod
    def interp(a, fa, fpa, b, fb, fpb, xmin, xmax, order):
        ymin, ymax = (xmin - a) / (b - a), (xmax - a) / (b - a)
        if ymin > ymax:
            ymin, ymax = ymax, ymin
        if order > 2 and not (fpb != fpa) and fpb != math.inf:
            fpa, fpb = fpa * (b - a), fpb * (b - a)
            eta = 3 * (fb - fa) - 2 * fpa - fpb
            xi = fpa + fpb - 2 * (fb - fa)
            c = [fa, fpa, eta, xi]
            pe = lambda y: ((c[3] * y + c[2]) * y + c[1]) * y + c[0]
            y, fmin = ymin, pe(ymin)
            if pe(ymax) < fmin:
                y, fmin = ymax, pe(ymax)
            qa, qb, qc = 3 * xi, 2 * eta, fpa
            roots = []
            if qa != 0:
                disc = qb * qb - 4 * qa * qc
                if disc >= 0:
                    s = math.sqrt(disc)
                    roots = sorted([(-qb - s) / (2 * qa), (-qb + s) / (2 * qa)])
            elif qb != 0:
                roots = [-qc / qb]
            for r in roots:
                if ymin < r < ymax and pe(r) < fmin:
                    y, fmin = r, pe(r)
        else:
            fpa = fpa * (b - a)
            fl = fa + ymin * (fpa + ymin * (fb - fa - fpa))
            fh = fa + ymax * (fpa + ymax * (fb - fa - fpa))
            c = 2 * (fb - fa - fpa)
            y, fmin = ymin, fl
            if fh < fmin:
                y, fmin = ymax, fh
            if c > a:  # PCL 1.8.1 as published
                z = -fpa / c
                if ymin < z < ymax:
                    fz = fa + z * (fpa + z * (fb - fa - fpa))
                    if fz < fmin:
                        y = z
        return a + y * (b - a)

    def line_search(self, alpha1):
        rho, sigma, order = self.rho, self.sigma, self.order
        f0, fp0 = self._fdf(0.0)
        alpha, aprev, faprev, fpaprev = alpha1, 0.0, f0, fp0
        a, b, fa, fb, fpa, fpb = 0.0, alpha, f0, 0.0, fp0, 0.0
        i = 0
        while True:
            i += 1
            if not i - 1 < self.iters:
                break
            falpha = self._f(alpha)
            if falpha > f0 + alpha * rho * fp0 or falpha >= faprev:
                a, fa, fpa, b, fb, fpb = aprev, faprev, fpaprev, alpha, falpha, math.nan
                break
            fpalpha = self._df(alpha)
            if abs(fpalpha) <= -sigma * fp0:
                return 0, alpha
            if fpalpha >= 0:
                a, fa, fpa, b, fb, fpb = alpha, falpha, fpalpha, aprev, faprev, fpaprev
                break
            delta = alpha - aprev
            nxt = self.interp(aprev, faprev, fpaprev, alpha, falpha, fpalpha, alpha + delta,
                              alpha + self.tau1 * delta, order)
            aprev, faprev, fpaprev, alpha = alpha, falpha, fpalpha, nxt
        while True:
            i += 1
            if not i - 1 < self.iters:
                break
            delta = b - a
            alpha = self.interp(a, fa, fpa, b, fb, fpb, a + self.tau2 * delta, b - self.tau3 * delta, order)
            falpha = self._f(alpha)
            if (a - alpha) * fpa <= np.finfo(np.float64).eps:
                return 1, None
            if falpha > f0 + rho * alpha * fp0 or falpha >= fa:
                b, fb, fpb = alpha, falpha, math.nan
            else:
                fpalpha = self._df(alpha)
                if abs(fpalpha) <= -sigma * fp0:
                    return 0, alpha
                if ((b - a) >= 0 and fpalpha >= 0) or ((b - a) <= 0 and fpalpha <= 0):
                    b, fb, fpb = a, fa, fpa
                a, fa, fpa = alpha, falpha, fpalpha
        return 0, 0.0

    def step(self, x):
        f0 = self.f
        if self.pnorm == 0.0 or self.g0norm == 0.0 or self.fp0 == 0:
            return 1, x
        if self.delta_f < 0:
            dl = max(-self.delta_f, 10 * np.finfo(np.float64).eps * abs(f0))
            alpha1 = min(1.0, 2.0 * dl / (-self.fp0))
        else:
            alpha1 = abs(self.step_size)
        st, alpha = self.line_search(alpha1)
        if st != 0:
            return st, x
        self._fdf(alpha)
        self.f, x, self.g = self.fa, self.xa.copy(), self.ga.copy()
        self.delta_f = self.f - f0
        dx0, dg0 = x - self.x0, self.g - self.g0
        dxg, dgg, dxdg = float(dx0 @ self.g), float(dg0 @ self.g), float(dx0 @ dg0)
        dgn = float(np.linalg.norm(dg0))
        if dxdg != 0:
            B = dxg / dxdg
            A = -(1.0 + dgn * dgn / dxdg) * B + dgg / dxdg
        else:
            A = B = 0.0
        self.p = -A * dx0 - B * dg0 + self.g
        self.g0, self.x0 = self.g.copy(), x.copy()
        self.g0norm = float(np.linalg.norm(self.g0))
        self.pnorm = float(np.linalg.norm(self.p))
        d = -1.0 if float(self.p @ self.g) > 0 else 1.0
        self.p = self.p * (d / self.pnorm)
        self.pnorm = float(np.linalg.norm(self.p))
        self.fp0 = float(self.p @ self.g0)
        self.xa, self.fkey, self.ga, self.gkey = self.x0.copy(), 0.0, self.g0.copy(), 0.0
        self.dfa, self.dfkey = float(self.ga @ self.p), 0.0
        return 0, x


def estimate(T, S, Q, M, max_inner=20):
    if len(S) < 4:
        return None, 0
    x = np.array([T[0, 3], T[1, 3], T[2, 3], math.atan2(T[2, 1], T[2, 2]), math.asin(-float(T[2, 0])),
                  math.atan2(T[1, 0], T[0, 0])], dtype=np.float64)
    fn = Functor(S, Q, M)
    b = BFGS(fn)
    b.init(x)
    inner, result = 0, -1
    while True:
        inner += 1
        result, x = b.step(x)
        if result:
            break
        result = 0 if np.linalg.norm(b.g) < 1e-2 else -1
        if not (result == -1 and inner < max_inner):
            break
    if result in (0, 1) or inner == max_inner:
        return apply_state(x), fn.calls
    return None, fn.calls


def gicp(src, tgt, max_iter=100, tf_eps=4e-3, rot_eps=2e-3, dmax=0.04, k=20, eps=1e-3):
    """Full GICP::computeTransformation with guess = I; returns (T, iterations, trace, cov_s, cov_t)."""
    src = src.astype(np.float32)
    tgt = tgt.astype(np.float32)
    cs, ct = covariances(src, k, eps), covariances(tgt, k, eps)
    Cs, Ct = full3(cs), full3(ct)
    T = np.eye(4, dtype=np.float32)
    it, trace, conv = 0, [], False
    thr = dmax * dmax
    prev = T.copy()
    while not conv:
        q = xform32(T, src)
        nn, d2 = knn_exact(tgt, q, 1)
        nn, d2 = nn[:, 0], d2[:, 0]
        ok = d2.astype(np.float64) < thr
        R = T.astype(np.float64)[:3, :3]
        A = R[None] @ Cs[ok] @ R.T[None] + Ct[nn[ok]]
        M = np.linalg.inv(A)
        prev = T.copy()
        Tn, _ = estimate(T, src[ok], tgt[nn[ok]], M)
        if Tn is None:
            break
        T = Tn
        ratio = np.full((4, 4), 1.0 / tf_eps)
        ratio[:3, :3] = 1.0 / rot_eps
        delta = float(np.max(ratio * np.abs(prev - T).astype(np.float64)))
        trace.append(T.copy())
        it += 1
        if it >= max_iter or delta < 1:
            conv = True
            prev = T.copy()
    return prev, it, trace, cs, ct


def main():
    from leica_point_cloud_processing_amd import synth

    out_dir = os.path.join(ROOT, "tests", "golden")
    os.makedirs(out_dir, exist_ok=True)
    src, tgt, Trot = synth.cube_fixture(os.path.join(out_dir, "cube.ply"))
    cases = {
        "k1_cube_testconfig": (src, tgt, dict(dmax=5.0, tf_eps=5e-4)),
        "k2_cube_defaults": (src, tgt, {}),
    }
    scan, cad, Tp = synth.scan_vs_cad(6000, 6000)
    cases["k3_part_6k"] = (scan, cad, {})
    for name, (s, t, kw) in cases.items():
        T, it, trace, cs, ct = gicp(s, t, **kw)
        q = xform32(np.eye(4, dtype=np.float32), s)
        nn, d2 = knn_exact(t.astype(np.float32), q, 1)
        dmax = kw.get("dmax", 0.04)
        corr = np.where(d2[:, 0].astype(np.float64) < dmax * dmax, nn[:, 0], -1).astype(np.int32)
        np.savez_compressed(
            os.path.join(out_dir, f"{name}.npz"),
            source=s.astype(np.float32), target=t.astype(np.float32),
            params=np.array([kw.get("dmax", 0.04), kw.get("tf_eps", 4e-3), 2e-3, 100, 20], np.float64),
            cov_source_head=cs[:256], cov_target_head=ct[:256],
            corr_identity=corr, final_T=T, iterations=np.int32(it),
            trace=np.array(trace, np.float32))
        print(name, "iterations", it, "\n", T)


if __name__ == "__main__":
    main()
