"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (oracle/libgicp_ref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline -- never as a compute path of the product.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libgicp_ref.so")


class RefParams(ctypes.Structure):
    _fields_ = [
        ("max_iterations", ctypes.c_int),
        ("transformation_epsilon", ctypes.c_double),
        ("rotation_epsilon", ctypes.c_double),
        ("max_corr_dist", ctypes.c_double),
        ("gicp_epsilon", ctypes.c_double),
        ("k_correspondences", ctypes.c_int),
        ("max_inner_iterations", ctypes.c_int),
        ("fixed_iterations", ctypes.c_int),
        ("threads", ctypes.c_int),
        ("objective", ctypes.c_int),
        ("solver", ctypes.c_int),
        ("variant", ctypes.c_int),
    ]


class RefResult(ctypes.Structure):
    _fields_ = [
        ("converged", ctypes.c_int),
        ("iterations", ctypes.c_int),
        ("n_corr_last", ctypes.c_int),
        ("n_evals", ctypes.c_int),
        ("t_cov_s", ctypes.c_double),
        ("t_loop_s", ctypes.c_double),
        ("t_total_s", ctypes.c_double),
    ]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    P, FP, DP, IP = ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)
    sz = ctypes.c_size_t
    sig = {
        "ref_default_params": (None, [ctypes.POINTER(RefParams)]),
        "ref_create": (P, [ctypes.POINTER(RefParams)]),
        "ref_destroy": (None, [P]),
        "ref_set_params": (ctypes.c_int, [P, ctypes.POINTER(RefParams)]),
        "ref_set_source": (ctypes.c_int, [P, P, sz, sz]),
        "ref_set_target": (ctypes.c_int, [P, P, sz, sz]),
        "ref_align": (ctypes.c_int, [P, FP, FP, ctypes.POINTER(RefResult), FP]),
        "ref_fitness": (ctypes.c_int, [P, FP, ctypes.c_double, DP]),
        "ref_covariances": (ctypes.c_int, [P, sz, sz, ctypes.c_int, ctypes.c_double, ctypes.c_int, DP]),
        "ref_knn": (ctypes.c_int, [P, sz, sz, P, sz, ctypes.c_int, IP, FP]),
        "ref_correspondences": (ctypes.c_int, [P, FP, FP, IP, FP, DP]),
        "ref_fdf": (ctypes.c_int, [P, DP, DP, DP]),
        "ref_moments": (ctypes.c_int, [P, FP, DP]),
        "ref_moments_range": (ctypes.c_int, [P, FP, ctypes.c_int, ctypes.c_int, DP]),
        "ref_fdf_sums": (ctypes.c_int, [P, DP, ctypes.c_int, ctypes.c_int, DP]),
        "ref_set_sum_order": (ctypes.c_int, [P, ctypes.c_int, P, sz]),
        "ref_fdf_mode_sums": (ctypes.c_int, [P, DP, DP]),
        "ref_set_mahalanobis_upper": (ctypes.c_int, [P, ctypes.c_int]),
        "ref_apply_state": (None, [DP, FP]),
        "ref_segment_differences": (ctypes.c_int, [P, sz, sz, P, sz, sz, ctypes.c_double, P, ctypes.POINTER(sz)]),
        "ref_voxel_grid": (ctypes.c_int, [P, sz, sz, ctypes.c_int, FP, ctypes.c_int, FP, P, ctypes.POINTER(sz),
                                          ctypes.POINTER(ctypes.c_int)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def cm(T: np.ndarray) -> np.ndarray:
    """numpy 4x4 -> column-major float32 buffer (Eigen storage)."""
    return np.ascontiguousarray(np.asarray(T, dtype=np.float32).T).reshape(16)


def from_cm(buf: np.ndarray) -> np.ndarray:
    return np.asarray(buf, dtype=np.float32).reshape(4, 4).T.copy()


class RefGICP:
    """PCL 1.8.1 GICP restatement with PCL's setter / align / fitness surface."""

    def __init__(self, max_iterations=100, transformation_epsilon=4e-3, rotation_epsilon=2e-3,
                 max_corr_dist=0.04, gicp_epsilon=1e-3, k=20, max_inner_iterations=20,
                 fixed_iterations=False, threads=1, objective=0, solver=0, variant=0):
        self.lib = load()
        self.p = RefParams()
        self.lib.ref_default_params(ctypes.byref(self.p))
        self.p.max_iterations = max_iterations
        self.p.transformation_epsilon = transformation_epsilon
        self.p.rotation_epsilon = rotation_epsilon
        self.p.max_corr_dist = max_corr_dist
        self.p.gicp_epsilon = gicp_epsilon
        self.p.k_correspondences = k
        self.p.max_inner_iterations = max_inner_iterations
        self.p.fixed_iterations = int(bool(fixed_iterations))
        self.p.threads = threads
        self.p.objective = objective
        self.p.solver = solver
        self.p.variant = variant
        self.h = self.lib.ref_create(ctypes.byref(self.p))
        self.ns = 0

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ref_destroy(self.h)
            self.h = None

    def set_params(self, **kw):
        for k, v in kw.items():
            setattr(self.p, k, v)
        self.lib.ref_set_params(self.h, ctypes.byref(self.p))

    def set_source(self, xyz):
        self._src = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        self.ns = len(self._src)
        return self.lib.ref_set_source(self.h, self._src.ctypes.data, self.ns, 12)

    def set_target(self, xyz):
        self._tgt = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        return self.lib.ref_set_target(self.h, self._tgt.ctypes.data, len(self._tgt), 12)

    def align(self, guess=None, want_trace=False):
        g = cm(np.eye(4) if guess is None else guess)
        out = np.zeros(16, np.float32)
        res = RefResult()
        trace = np.zeros(16 * max(1, self.p.max_iterations), np.float32) if want_trace else None
        rc = self.lib.ref_align(self.h, _fp(g), _fp(out), ctypes.byref(res), _fp(trace) if want_trace else None)
        info = {k: getattr(res, k) for k, _ in RefResult._fields_}
        info["rc"] = rc
        if want_trace:
            it = res.iterations
            info["trace"] = [from_cm(trace[16 * i:16 * i + 16]) for i in range(it)]
        return from_cm(out), info

    def fitness(self, T, max_range=np.finfo(np.float64).max):
        out = ctypes.c_double()
        rc = self.lib.ref_fitness(self.h, _fp(cm(T)), max_range, ctypes.byref(out))
        assert rc == 0
        return out.value

    def correspondences(self, T, guess=None):
        n = self.ns
        tgt = np.zeros(n, np.int32)
        d2 = np.zeros(n, np.float32)
        M = np.zeros((n, 9), np.float64)
        g = cm(np.eye(4) if guess is None else guess)
        m = self.lib.ref_correspondences(self.h, _fp(cm(T)), _fp(g), _ip(tgt), _fp(d2), _dp(M))
        return m, tgt, d2, M

    def set_sum_order(self, mode: int, perm=None):
        """r06 summation-order ledger (gicp_ref.h ref_set_sum_order): 0 default, 1 the engine's fixed tree
        over the stream order `perm` (source indices), 2 reversed sequential, 3 sequential over `perm`."""
        buf = None if perm is None else np.ascontiguousarray(perm, np.uint32)
        rc = self.lib.ref_set_sum_order(self.h, int(mode), None if buf is None else buf.ctypes.data,
                                        0 if buf is None else len(buf))
        assert rc == 0, rc
        self._sum_perm = buf

    def set_mahalanobis_upper(self, on: bool):
        """gicp_ref.h ref_set_mahalanobis_upper: mirror M's upper triangle (the engine's storage)"""
        assert self.lib.ref_set_mahalanobis_upper(self.h, int(bool(on))) == 0

    def fdf_mode_sums(self, x):
        """raw 14 sums of one pass at x in the current summation mode (set_sum_order)"""
        x = np.asarray(x, np.float64)
        out = np.zeros(14, np.float64)
        assert self.lib.ref_fdf_mode_sums(self.h, _dp(x), _dp(out)) == 0
        return out

    def fdf_sums(self, x, c0, c1):
        x = np.asarray(x, np.float64)
        out = np.zeros(14, np.float64)
        rc = self.lib.ref_fdf_sums(self.h, _dp(x), int(c0), int(c1), _dp(out))
        assert rc == 0
        return out

    def moments(self, T0):
        out = np.zeros(74, np.float64)
        rc = self.lib.ref_moments(self.h, _fp(cm(T0)), _dp(out))
        assert rc == 0
        return out

    def moments_range(self, T0, c0, c1):
        out = np.zeros(74, np.float64)
        rc = self.lib.ref_moments_range(self.h, _fp(cm(T0)), int(c0), int(c1), _dp(out))
        assert rc == 0
        return out

    def fdf(self, x):
        x = np.asarray(x, np.float64)
        f = ctypes.c_double()
        g = np.zeros(6, np.float64)
        rc = self.lib.ref_fdf(self.h, _dp(x), ctypes.byref(f), _dp(g))
        assert rc == 0
        return f.value, g


def covariances(xyz, k=20, eps=1e-3, threads=1) -> np.ndarray:
    lib = load()
    xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
    out = np.zeros((len(xyz), 6), np.float64)
    rc = lib.ref_covariances(xyz.ctypes.data, len(xyz), 12, k, eps, threads, _dp(out))
    if rc != 0:
        raise ValueError(f"ref_covariances rc={rc}")
    return out


def knn(xyz, queries, k):
    lib = load()
    xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
    q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, 3)
    idx = np.zeros((len(q), k), np.int32)
    d2 = np.zeros((len(q), k), np.float32)
    lib.ref_knn(xyz.ctypes.data, len(xyz), 12, q.ctypes.data, len(q), k, _ip(idx), _fp(d2))
    return idx, d2


def apply_state(x) -> np.ndarray:
    lib = load()
    x = np.asarray(x, np.float64)
    out = np.zeros(16, np.float32)
    lib.ref_apply_state(_dp(x), _fp(out))
    return from_cm(out)


def _records(a):
    """(owner, pointer, n, stride) of an (n, 3) xyz array or an n-record structured array."""
    a = np.ascontiguousarray(a)
    if a.dtype.names:
        return a, a.ctypes.data, len(a), a.dtype.itemsize
    a = np.ascontiguousarray(a, dtype=np.float32).reshape(-1, 3)
    return a, a.ctypes.data, len(a), 12


def segment_differences(cloud_in, cloud_sub, sqr_threshold):
    """pcl::getPointCloudDifference restatement: (keep mask, kept count)."""
    lib = load()
    a, pa, n, sa = _records(cloud_in)
    b, pb, ns, sb = _records(cloud_sub)
    keep = np.zeros(max(n, 1), np.uint8)
    cnt = ctypes.c_size_t()
    rc = lib.ref_segment_differences(pa, n, sa, pb, ns, sb, float(sqr_threshold), keep.ctypes.data, ctypes.byref(cnt))
    assert rc == 0
    return keep[:n].astype(bool), int(cnt.value)


def voxel_grid(records, leaf, min_points=0, rgb_offset=16):
    """pcl::VoxelGrid<PointXYZRGB> restatement over an n-record array (rgb word at rgb_offset,
    -1 for none): (xyz (m, 3) float32, rgba (m,) uint32, overflow flag)."""
    lib = load()
    a, pa, n, stride = _records(records)
    if not a.dtype.names:
        rgb_offset = -1
    leaf = np.broadcast_to(np.asarray(leaf, np.float32), (3,)).copy()
    xyz = np.zeros((max(n, 1), 3), np.float32)
    rgba = np.zeros(max(n, 1), np.uint32)
    nout = ctypes.c_size_t()
    ovf = ctypes.c_int()
    rc = lib.ref_voxel_grid(pa, n, stride, rgb_offset, _fp(leaf), int(min_points), _fp(xyz), rgba.ctypes.data,
                            ctypes.byref(nout), ctypes.byref(ovf))
    assert rc == 0
    m = nout.value
    return xyz[:m].copy(), rgba[:m].copy(), bool(ovf.value)
