"""GICPEngine: the MI355X GICP behind pcl::GeneralizedIterativeClosestPoint's API surface.

Mirrors the subset of pcl::GeneralizedIterativeClosestPoint<PointXYZRGB,PointXYZRGB> that
GICPAlignment uses (/root/reference/src/GICPAlignment.cpp:48-54, 89-105, 116-123):
setMaximumIterations, setMaxCorrespondenceDistance, setTransformationEpsilon,
setRANSACOutlierRejectionThreshold (stored, unused by GICP), setInputSource, setInputTarget,
align, hasConverged, getFinalTransformation, getFitnessScore, getMaximumIterations.
All compute goes through libmgicp.so (include/mi355x_gicp.h); nothing runs on the CPU.
"""
from __future__ import annotations

import atexit
import ctypes

import numpy as np

from . import _lib
from .cloud import PointCloudRGB

DBL_MAX = float(np.finfo(np.float64).max)
_LIVE: set = set()
_SHUTTING_DOWN = [False]


@atexit.register
def _mark_shutdown():
    _SHUTTING_DOWN[0] = True


def _cm(T) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(T, dtype=np.float32).T).reshape(16)


def _from_cm(buf) -> np.ndarray:
    return np.asarray(buf, dtype=np.float32).reshape(4, 4).T.copy()


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class GICPEngine:
    # mgicp_debug_option forms applied to every new engine before its own `options` (the GPU test suite
    # sets {"target_cache": 0} so engines of different tests never adopt each other's targets)
    DEFAULT_OPTIONS: dict = {}

    def __init__(self, device: int = -1, options: dict | None = None, **params):
        """params: mgicp_params fields; options: mgicp_debug_option forms (tests / diagnostics only)"""
        self._lib = _lib.load()
        self.params = _lib.default_params()
        self.params.device = device
        for k, v in params.items():
            setattr(self.params, k, v)
        h = ctypes.c_void_p()
        rc = self._lib.mgicp_create(ctypes.byref(h), ctypes.byref(self.params))
        if rc != 0:
            raise _lib.MgicpError(rc, "mgicp_create failed (no HIP device or invalid parameters)")
        self._h = h
        _LIVE.add(id(self))
        self.ransac_outlier_threshold = 0.05
        self._input = None
        self._converged = False
        self._final = np.eye(4, dtype=np.float32)
        self.last_result = None
        for k, v in {**GICPEngine.DEFAULT_OPTIONS, **(options or {})}.items():
            self.debug_option(k, v)

    def cache_stats(self) -> dict:
        """The process-wide target cache (mgicp_debug_cache_stats)."""
        out = (ctypes.c_longlong * 5)()
        self._check(self._lib.mgicp_debug_cache_stats(self._h, out), "cache_stats")
        return {"adopted": int(out[0]), "hits": int(out[1]), "donations": int(out[2]), "cached": int(out[3]),
                "source_spec": ("none", "pending", "kept", "discarded")[int(out[4])]}

    @staticmethod
    def release_cache():
        """Free the process-wide target cache (mgicp_release_cache)."""
        _lib.load().mgicp_release_cache()

    def debug_option(self, name: str, value):
        """mgicp_debug_option: a test / diagnostic form of the engine on this context only"""
        self._check(self._lib.mgicp_debug_option(self._h, name.encode(), float(value)), f"debug option {name}")

    def close(self):
        """Release the device context (deterministically, before interpreter shutdown)."""
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            _LIVE.discard(id(self))
            self._lib.mgicp_destroy(h)

    def __del__(self):
        # at interpreter shutdown the HIP runtime may already be torn down: leave the context
        # to the process exit instead of racing the runtime's own destructors
        if not _SHUTTING_DOWN[0]:
            self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- helpers -------------------------------------------------------------------------
    def _check(self, rc: int, what: str):
        if rc < 0:
            raise _lib.MgicpError(rc, f"{what}: {self._lib.mgicp_last_error(self._h).decode()}")
        return rc

    def _push_params(self):
        self._check(self._lib.mgicp_set_params(self._h, ctypes.byref(self.params)), "mgicp_set_params")

    # -- pcl::Registration setters -----------------------------------------------------------
    def setMaximumIterations(self, n: int):
        self.params.max_iter = int(n)
        self._push_params()

    def getMaximumIterations(self) -> int:
        return int(self.params.max_iter)

    def setMaxCorrespondenceDistance(self, d: float):
        self.params.max_corr_dist = float(d)
        self._push_params()

    def setTransformationEpsilon(self, eps: float):
        self.params.tf_eps = float(eps)
        self._push_params()

    def setRotationEpsilon(self, eps: float):
        self.params.rot_eps = float(eps)
        self._push_params()

    def setSolver(self, solver: int):
        """MGICP_SOLVER_PCL_BFGS (default, PCL 1.8.1 trajectory) or MGICP_SOLVER_GN (fast mode).
        Grids and covariances stay cached (PCL's dirty-flag semantics)."""
        self.params.solver = int(solver)
        self._push_params()

    def setRANSACOutlierRejectionThreshold(self, th: float):
        self.ransac_outlier_threshold = float(th)  # stored; GICP never uses it (PCL 1.8.1)

    def setInputSource(self, cloud):
        self._input = cloud
        keep, ptr, n, stride = self._cloud_arg(cloud)
        self._check(self._lib.mgicp_set_source(self._h, ptr, n, stride), "setInputSource")

    def setInputTarget(self, cloud):
        keep, ptr, n, stride = self._cloud_arg(cloud)
        self._check(self._lib.mgicp_set_target(self._h, ptr, n, stride), "setInputTarget")

    @staticmethod
    def _cloud_arg(cloud):
        """(owner, pointer, n, stride); `owner` keeps a converted copy alive across the call."""
        if isinstance(cloud, PointCloudRGB):
            return (cloud,) + cloud.ctypes_xyz()
        a = np.ascontiguousarray(cloud, dtype=np.float32).reshape(-1, 3)
        return a, a.ctypes.data, len(a), 12

    def set_source_xyz(self, xyz):
        self._src_keep = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        self._input = None
        self._check(self._lib.mgicp_set_source(self._h, self._src_keep.ctypes.data, len(self._src_keep), 12),
                    "set_source")

    def set_target_xyz(self, xyz):
        self._tgt_keep = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        self._check(self._lib.mgicp_set_target(self._h, self._tgt_keep.ctypes.data, len(self._tgt_keep), 12),
                    "set_target")

    def set_source_device(self, ptr: int, n: int, stride: int):
        self._input = None
        self._check(self._lib.mgicp_set_source_device(self._h, ctypes.c_void_p(ptr), n, stride), "set_source_device")

    def set_target_device(self, ptr: int, n: int, stride: int):
        self._check(self._lib.mgicp_set_target_device(self._h, ctypes.c_void_p(ptr), n, stride), "set_target_device")

    # -- the hot path ----------------------------------------------------------------------
    def align(self, output: PointCloudRGB | None = None, guess=None) -> np.ndarray:
        """Registration::align(output, guess).  Returns getFinalTransformation()."""
        g = _cm(guess) if guess is not None else None
        out = np.zeros(16, np.float32)
        res = _lib.MgicpResult()
        rc = self._lib.mgicp_align(self._h, _fp(g) if g is not None else None, _fp(out), ctypes.byref(res))
        self.last_result = {k: getattr(res, k) for k, _ in _lib.MgicpResult._fields_}
        if rc == _lib.MGICP_E_SOLVER:
            self._converged = False  # PCL catches the solver exception; converged_ stays false
        else:
            self._check(rc, "align")
            self._converged = bool(res.converged)
        self._final = _from_cm(out)
        if output is not None and isinstance(self._input, PointCloudRGB):
            # output = transformPointCloud(*input_, output, final_transformation_)
            output.copy_from(self._input)
            self.transform_source_into(self._final, output)
        return self._final

    def hasConverged(self) -> bool:
        return self._converged

    def getFinalTransformation(self) -> np.ndarray:
        return self._final.copy()

    def getFitnessScore(self, max_range: float = DBL_MAX) -> float:
        out = ctypes.c_double()
        self._check(self._lib.mgicp_fitness(self._h, _fp(_cm(self._final)), max_range, ctypes.byref(out)),
                    "getFitnessScore")
        return out.value

    def fitness(self, T, max_range: float = DBL_MAX) -> float:
        out = ctypes.c_double()
        self._check(self._lib.mgicp_fitness(self._h, _fp(_cm(T)), max_range, ctypes.byref(out)), "fitness")
        return out.value

    def transform_source_into(self, T, cloud: PointCloudRGB):
        """xyz of `cloud` := T * source (device kernel; `cloud` must have the source's size)."""
        ptr, n, stride = cloud.ctypes_xyz()
        self._check(self._lib.mgicp_transform_source(self._h, _fp(_cm(T)), ctypes.c_void_p(ptr), stride),
                    "transform_source")

    def transform_cloud(self, T, cloud_in: PointCloudRGB, cloud_out: PointCloudRGB) -> None:
        """pcl::transformPointCloud(cloud_in, cloud_out, T) with the xyz transform on the GPU."""
        if cloud_out is not cloud_in:
            cloud_out.copy_from(cloud_in)
        _, ptr, n, stride = self._cloud_arg(cloud_out)
        self._check(self._lib.mgicp_transform_cloud(self._h, _fp(_cm(T)), ctypes.c_void_p(ptr), n, stride,
                                                    ctypes.c_void_p(ptr), stride), "transform_cloud")

    # -- helpers of GICPAlignment(use_covariances=true) --------------------------------------
    def cloud_resolution(self, cloud) -> float:
        """Utils::computeCloudResolution on the GPU (mean distance to the nearest other point)."""
        keep, ptr, n, stride = self._cloud_arg(cloud)
        out = ctypes.c_double()
        self._check(self._lib.mgicp_cloud_resolution(self._h, ctypes.c_void_p(ptr), n, stride, ctypes.byref(out)),
                    "cloud_resolution")
        return out.value

    def radius_filter(self, cloud, radius: float, min_neighbors: int = 3) -> np.ndarray:
        """bool mask: >= min_neighbors points (self included) within `radius` (NormalEstimation's
        non-NaN condition)."""
        keep, ptr, n, stride = self._cloud_arg(cloud)
        keep = np.zeros(n, np.uint8)
        self._check(self._lib.mgicp_radius_filter(self._h, ctypes.c_void_p(ptr), n, stride, float(radius),
                                                  int(min_neighbors), keep.ctypes.data), "radius_filter")
        return keep.astype(bool)

    # -- FOD-side callers ------------------------------------------
    def segment_differences(self, cloud_in, cloud_sub, sqr_threshold: float, T=None):
        """pcl::SegmentDifferences (Filter::removeFromCloud): bool keep mask over cloud_in (after T)
        and the kept count."""
        keep_in, pin, n, sin_ = self._cloud_arg(cloud_in)
        keep_sub, psub, ns, ssub = self._cloud_arg(cloud_sub)
        keep = np.zeros(max(n, 1), np.uint8)
        cnt = ctypes.c_size_t()
        tcm = _cm(T) if T is not None else None
        self._check(self._lib.mgicp_segment_differences(
            self._h, _fp(tcm) if tcm is not None else None, ctypes.c_void_p(pin), n, sin_, ctypes.c_void_p(psub),
            ns, ssub, float(sqr_threshold), keep.ctypes.data, ctypes.byref(cnt)), "segment_differences")
        return keep[:n].astype(bool), int(cnt.value)

    def voxel_grid(self, cloud: PointCloudRGB, leaf, min_points_per_voxel: int = 0) -> PointCloudRGB:
        """pcl::VoxelGrid<PointXYZRGB>::filter (Filter::downsampleCloud) -> a new cloud."""
        from .cloud import POINT_XYZRGB

        leaf = np.broadcast_to(np.asarray(leaf, np.float64), (3,)).copy()
        _, ptr, n, stride = self._cloud_arg(cloud)
        out = PointCloudRGB()
        out.points = np.empty(max(n, 1), dtype=POINT_XYZRGB)  # capacity; the call writes n_out whole records
        nout = ctypes.c_size_t()
        self._check(self._lib.mgicp_voxel_grid(
            self._h, ctypes.c_void_p(ptr), n, stride, int(POINT_XYZRGB.fields["rgb"][1]), _dp(leaf),
            int(min_points_per_voxel), out.points.ctypes.data, POINT_XYZRGB.itemsize, ctypes.byref(nout)),
            "voxel_grid")
        out.points = out.points[:nout.value].copy()
        return out

    # -- multi-GPU ------------------------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        rc = _lib.load().mgicp_get_unique_id(buf)
        if rc != 0:
            raise _lib.MgicpError(rc, "mgicp_get_unique_id")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes | None):
        buf = ctypes.create_string_buffer(uid, 128) if uid is not None else None
        self._check(self._lib.mgicp_comm_init(self._h, nranks, rank, buf), "comm_init")

    def attach_shm(self, name: str, max_source_points: int = 0):
        """Node-local transport of the per-pass sums (every rank, same name): the GPUs write their
        super rows into one shared-memory segment, every host takes the same fixed-order total."""
        self._check(self._lib.mgicp_comm_attach_shm(self._h, name.encode(), int(max_source_points)),
                    "comm_attach_shm")

    def attach_xgmi(self, on: bool = True):
        """per-pass super rows over xGMI (peer device memory) after attach_shm (mgicp_comm_attach_xgmi)"""
        self._check(self._lib.mgicp_comm_attach_xgmi(self._h, int(bool(on))), "mgicp_comm_attach_xgmi")

    def detach_shm(self):
        """Back to the previous transport (RCCL or local)."""
        self._check(self._lib.mgicp_comm_attach_shm(self._h, None, 0), "comm_attach_shm(detach)")

    PASS_STATS = ("server_launches", "server_passes", "launched_passes", "takeovers", "bar_commands",
                  "row_allocs", "transport", "server_denied")

    def pass_stats(self) -> dict:
        """Objective-pass path counters (mgicp_debug_pass_stats)."""
        out = (ctypes.c_longlong * 8)()
        self._check(self._lib.mgicp_debug_pass_stats(self._h, out), "pass_stats")
        return {k: int(out[i]) for i, k in enumerate(self.PASS_STATS)}

    def server_time(self, reset: bool = False) -> dict:
        """The resident pass server as the aligns run it (mgicp_debug_server_time): summed launch
        duration, passes and launches since the last reset; ms_per_pass = the in-align pass."""
        ms = ctypes.c_double()
        passes = ctypes.c_longlong()
        launches = ctypes.c_longlong()
        self._check(self._lib.mgicp_debug_server_time(self._h, ctypes.byref(ms), ctypes.byref(passes),
                                                      ctypes.byref(launches), int(reset)), "server_time")
        p = int(passes.value)
        return {"ms": ms.value, "passes": p, "launches": int(launches.value),
                "ms_per_pass": ms.value / p if p else None}

    def debug_target_cov_slice(self, nranks: int, rank: int, n_target: int) -> np.ndarray:
        """slice `rank` of `nranks` of the target covariances as an N-rank context computes it before
        its all-gather (mgicp_debug_target_cov_slice)"""
        out = np.zeros((max(1, -(-n_target // nranks)), 6), np.float64)
        cnt = self._check(self._lib.mgicp_debug_target_cov_slice(self._h, int(nranks), int(rank), _dp(out)),
                          "debug_target_cov_slice")
        return out[:cnt].copy()

    VLIST_STATS = ("requested", "pending", "lists", "entries", "reject", "overflow", "pool_used", "cells")

    def vlist_stats(self) -> dict:
        """The target's 1-NN cell lists (mgicp_debug_vlist_stats)."""
        out = (ctypes.c_longlong * 8)()
        self._check(self._lib.mgicp_debug_vlist_stats(self._h, out), "vlist_stats")
        return {k: int(out[i]) for i, k in enumerate(self.VLIST_STATS)}

    # -- introspection (parity tests, profiling) ----------------------------------------------
    def debug_source_order(self, n: int) -> np.ndarray:
        """Original indices of the source points in the objective's stream order (mgicp_debug_source_order)."""
        out = np.zeros(n, np.uint32)
        m = self._check(self._lib.mgicp_debug_source_order(self._h, out.ctypes.data, n), "debug_source_order")
        return out[:m]

    def debug_covariances(self, which: str, n: int) -> np.ndarray:
        out = np.zeros((n, 6), np.float64)
        self._check(self._lib.mgicp_debug_covariances(self._h, 0 if which == "source" else 1, _dp(out)),
                    "debug_covariances")
        return out

    def debug_correspondences(self, T, n: int):
        tgt = np.full(n, -1, np.int32)
        M = np.zeros((n, 6), np.float64)
        m = self._check(self._lib.mgicp_debug_correspondences(
            self._h, _fp(_cm(T)), tgt.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _dp(M)), "debug_correspondences")
        return m, tgt, M

    def debug_correspondences_seeded(self, T, n: int):
        """The same sweep seeded with the previous sweep's matches (outer iterations >= 2)."""
        tgt = np.full(n, -1, np.int32)
        M = np.zeros((n, 6), np.float64)
        m = self._check(self._lib.mgicp_debug_correspondences_seeded(
            self._h, _fp(_cm(T)), tgt.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _dp(M)),
            "debug_correspondences_seeded")
        return m, tgt, M

    def debug_fdf(self, x):
        x = np.asarray(x, np.float64)
        f = ctypes.c_double()
        g = np.zeros(6, np.float64)
        self._check(self._lib.mgicp_debug_fdf(self._h, _dp(x), ctypes.byref(f), _dp(g)), "debug_fdf")
        return f.value, g

    def debug_fdf_sums(self, x) -> np.ndarray:
        x = np.asarray(x, np.float64)
        out = np.zeros(16, np.float64)
        self._check(self._lib.mgicp_debug_fdf_sums(self._h, _dp(x), _dp(out)), "debug_fdf_sums")
        return out

    def debug_wave_reduce(self, vals) -> tuple:
        """(shuffle-tree sums, reduce-scatter sums) of vals[w][64][16] per wave w (the chunk reduction)"""
        vals = np.ascontiguousarray(vals, np.float64)
        nw = vals.shape[0]
        assert vals.shape == (nw, 64, 16)
        tree = np.zeros((nw, 16), np.float64)
        rs = np.zeros((nw, 16), np.float64)
        self._check(self._lib.mgicp_debug_wave_reduce(self._h, _dp(vals), int(nw), _dp(tree), _dp(rs)),
                    "debug_wave_reduce")
        return tree, rs

    def debug_pass_bench(self, x, npasses: int, mode: int = 0):
        """(ms per pass, sums of the last pass): npasses objective passes at x over the last sweep,
        back to back (mode 0: the resident pass server, 1: one launch per pass), HIP-event timed"""
        x = np.asarray(x, np.float64)
        ms = ctypes.c_double()
        out = np.zeros(16, np.float64)
        self._check(self._lib.mgicp_debug_pass_bench(self._h, _dp(x), int(npasses), int(mode), ctypes.byref(ms),
                                                     _dp(out)), "debug_pass_bench")
        return ms.value, out

    def debug_trace(self, max_iters: int = 1000):
        buf = np.zeros(16 * max_iters, np.float32)
        n = self._check(self._lib.mgicp_debug_trace(self._h, _fp(buf), max_iters), "debug_trace")
        return [_from_cm(buf[16 * i:16 * i + 16]) for i in range(min(n, max_iters))]

    def set_profiling(self, on: bool):
        self._check(self._lib.mgicp_set_profiling(self._h, int(on)), "set_profiling")

    def debug_moments(self, T) -> np.ndarray:
        """MGICP_SOLVER_GN's 74 moments (+ pad) at T over the last correspondence sweep."""
        out = np.zeros(80, np.float64)
        self._check(self._lib.mgicp_debug_moments(self._h, _fp(_cm(T)), _dp(out)), "debug_moments")
        return out

    def debug_supers(self, kind: str, arg) -> np.ndarray:
        """This shard's super partials of one pass of the fixed reduction tree: kind "fdf" (arg = x),
        "moments" (arg = T) or "fitness" (arg = (T, max_range)); shape (nsup_local, 16 or 80)."""
        if kind == "fdf":
            k, a, nv = 0, np.asarray(arg, np.float64), 16
        elif kind == "moments":
            k, a, nv = 1, np.asarray(_cm(arg), np.float64), 80
        elif kind == "fitness":
            T, max_range = arg
            k, a, nv = 2, np.concatenate([np.asarray(_cm(T), np.float64), [float(max_range)]]), 16
        else:
            raise ValueError(kind)
        cap = 1 << 16
        out = np.zeros((cap, nv), np.float64)
        n = self._check(self._lib.mgicp_debug_supers(self._h, k, _dp(np.ascontiguousarray(a)), _dp(out), cap),
                        "debug_supers")
        return out[:n].copy()

    def debug_finish_supers(self, rows: np.ndarray, nsup: int, maxsup: int, nranks: int) -> np.ndarray:
        """The multi-GPU finish: fixed-order total of nsup supers held as nranks rows of maxsup."""
        rows = np.ascontiguousarray(rows, np.float64)
        nv = rows.shape[-1]
        out = np.zeros(nv, np.float64)
        self._check(self._lib.mgicp_debug_finish_supers(self._h, nv, _dp(rows), nsup, maxsup, nranks, _dp(out)),
                    "debug_finish_supers")
        return out

    def kernel_times(self):
        nf = _lib.MGICP_KERNEL_FAMILIES
        ms = np.zeros(nf, np.float64)
        cnt = np.zeros(nf, np.int32)
        self._check(self._lib.mgicp_debug_kernel_times(self._h, _dp(ms), cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_int))),
                    "kernel_times")
        names = ["knn_cov", "correspond", "fdf", "reduce_finish", "compact", "gn_moments"]
        return {names[i]: {"avg_ms": float(ms[i]), "count": int(cnt[i])} for i in range(nf)}
