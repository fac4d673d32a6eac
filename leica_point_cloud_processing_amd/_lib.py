"""ctypes binding of libmgicp.so (include/mi355x_gicp.h).

The HIP engine is the only compute path of this package: if the in-tree library is missing
or cannot be loaded, every entry point raises immediately -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, os.environ.get("MGICP_LIB_NAME", "libmgicp.so"))  # variant builds for A/B
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "mi355x_gicp.h")

MGICP_OK = 0
MGICP_E_INVALID = -1
MGICP_E_TOO_FEW_POINTS = -2
MGICP_E_SOLVER = -3
MGICP_E_NONFINITE = -4
MGICP_E_HIP = -5
MGICP_E_COMM = -6
MGICP_E_NOMEM = -7

MGICP_SOLVER_PCL_BFGS = 0
MGICP_SOLVER_GN = 1
MGICP_KERNEL_FAMILIES = 6


class MgicpParams(ctypes.Structure):
    _fields_ = [
        ("max_iter", ctypes.c_int),
        ("tf_eps", ctypes.c_double),
        ("rot_eps", ctypes.c_double),
        ("max_corr_dist", ctypes.c_double),
        ("gicp_eps", ctypes.c_double),
        ("k", ctypes.c_int),
        ("max_inner_iter", ctypes.c_int),
        ("solver", ctypes.c_int),
        ("device", ctypes.c_int),
        ("fixed_iterations", ctypes.c_int),
    ]


class MgicpResult(ctypes.Structure):
    _fields_ = [
        ("converged", ctypes.c_int),
        ("iterations", ctypes.c_int),
        ("n_corr", ctypes.c_int),
        ("n_evals", ctypes.c_int),
        ("ms_total", ctypes.c_double),
        ("ms_upload", ctypes.c_double),
        ("ms_prep", ctypes.c_double),
        ("ms_loop", ctypes.c_double),
    ]


class MgicpError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mgicp error {code}: {msg}")
        self.code = code


_P = ctypes.c_void_p
_FP = ctypes.POINTER(ctypes.c_float)
_DP = ctypes.POINTER(ctypes.c_double)
_IP = ctypes.POINTER(ctypes.c_int)
_SZ = ctypes.c_size_t

_SIGNATURES = {
    "mgicp_default_params": (None, [ctypes.POINTER(MgicpParams)]),
    "mgicp_create": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(MgicpParams)]),
    "mgicp_set_params": (ctypes.c_int, [_P, ctypes.POINTER(MgicpParams)]),
    "mgicp_last_error": (ctypes.c_char_p, [_P]),
    "mgicp_destroy": (None, [_P]),
    "mgicp_device_count": (ctypes.c_int, [_IP]),
    "mgicp_set_target": (ctypes.c_int, [_P, _P, _SZ, _SZ]),
    "mgicp_set_source": (ctypes.c_int, [_P, _P, _SZ, _SZ]),
    "mgicp_set_target_device": (ctypes.c_int, [_P, _P, _SZ, _SZ]),
    "mgicp_set_source_device": (ctypes.c_int, [_P, _P, _SZ, _SZ]),
    "mgicp_align": (ctypes.c_int, [_P, _FP, _FP, ctypes.POINTER(MgicpResult)]),
    "mgicp_fitness": (ctypes.c_int, [_P, _FP, ctypes.c_double, _DP]),
    "mgicp_transform_source": (ctypes.c_int, [_P, _FP, _P, _SZ]),
    "mgicp_transform_cloud": (ctypes.c_int, [_P, _FP, _P, _SZ, _SZ, _P, _SZ]),
    "mgicp_cloud_resolution": (ctypes.c_int, [_P, _P, _SZ, _SZ, _DP]),
    "mgicp_radius_filter": (ctypes.c_int, [_P, _P, _SZ, _SZ, ctypes.c_double, ctypes.c_int, _P]),
    "mgicp_segment_differences": (ctypes.c_int, [_P, _FP, _P, _SZ, _SZ, _P, _SZ, _SZ, ctypes.c_double, _P,
                                                  ctypes.POINTER(_SZ)]),
    "mgicp_voxel_grid": (ctypes.c_int, [_P, _P, _SZ, _SZ, ctypes.c_int, _DP, ctypes.c_int, _P, _SZ,
                                         ctypes.POINTER(_SZ)]),
    "mgicp_get_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "mgicp_comm_init": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]),
    "mgicp_comm_attach_shm": (ctypes.c_int, [_P, ctypes.c_char_p, _SZ]),
    "mgicp_comm_attach_xgmi": (ctypes.c_int, [_P, ctypes.c_int]),
    "mgicp_debug_pass_stats": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_longlong)]),
    "mgicp_debug_server_time": (ctypes.c_int, [_P, _DP, ctypes.POINTER(ctypes.c_longlong),
                                               ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]),
    "mgicp_debug_target_cov_slice": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _DP]),
    "mgicp_debug_vlist_stats": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_longlong)]),
    "mgicp_debug_source_order": (ctypes.c_int, [_P, ctypes.c_void_p, ctypes.c_size_t]),
    "mgicp_debug_covariances": (ctypes.c_int, [_P, ctypes.c_int, _DP]),
    "mgicp_debug_correspondences": (ctypes.c_int, [_P, _FP, _IP, _DP]),
    "mgicp_debug_correspondences_seeded": (ctypes.c_int, [_P, _FP, _IP, _DP]),
    "mgicp_debug_fdf": (ctypes.c_int, [_P, _DP, _DP, _DP]),
    "mgicp_debug_fdf_sums": (ctypes.c_int, [_P, _DP, _DP]),
    "mgicp_debug_pass_bench": (ctypes.c_int, [_P, _DP, ctypes.c_int, ctypes.c_int, _DP, _DP]),
    "mgicp_debug_moments": (ctypes.c_int, [_P, _FP, _DP]),
    "mgicp_debug_supers": (ctypes.c_int, [_P, ctypes.c_int, _DP, _DP, ctypes.c_int]),
    "mgicp_debug_finish_supers": (ctypes.c_int, [_P, ctypes.c_int, _DP, ctypes.c_longlong, ctypes.c_longlong,
                                                 ctypes.c_int, _DP]),
    "mgicp_debug_wave_reduce": (ctypes.c_int, [_P, _DP, ctypes.c_int, _DP, _DP]),
    "mgicp_debug_trace": (ctypes.c_int, [_P, _FP, ctypes.c_int]),
    "mgicp_debug_kernel_times": (ctypes.c_int, [_P, _DP, _IP]),
    "mgicp_set_profiling": (ctypes.c_int, [_P, ctypes.c_int]),
    "mgicp_debug_option": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_double]),
    "mgicp_debug_cache_stats": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_longlong)]),
    "mgicp_release_cache": (None, []),
}

_lib = None


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function declared in include/mi355x_gicp.h."""
    with open(path) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(mgicp_[a-z_0-9]+)\s*\(", text)))


def _mapped_hip_runtimes() -> set[str]:
    """Real paths of every HIP runtime (libamdhip64*) mapped into this process."""
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) == 6 and "libamdhip64" in os.path.basename(parts[5].strip()):
                    out.add(os.path.realpath(parts[5].strip()))
    except OSError:  # no procfs: nothing to check against
        pass
    return out


def _rocm_lib_dir() -> str:
    return os.path.realpath(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib"))


def check_single_hip_runtime(when: str) -> None:
    """libmgicp.so links ROCm's HIP runtime (/opt/rocm/lib/libamdhip64.so.7).  A second HIP runtime
    in the same process -- torch bundles its own (torch/lib/libamdhip64.so, a different ROCm
    release) and maps it at `import torch` -- was observed to corrupt the heap on MI355X ("double
    free or corruption" at teardown, round 1, parallel.py).  Refuse that combination loudly."""
    libs = _mapped_hip_runtimes()
    foreign = sorted(p for p in libs if os.path.dirname(p) != _rocm_lib_dir())
    if foreign or len(libs) > 1:
        raise MgicpError(
            MGICP_E_HIP,
            f"{when}: another HIP runtime is mapped in this process ({', '.join(sorted(libs))}); libmgicp.so "
            f"uses {_rocm_lib_dir()}/libamdhip64.so and two HIP runtimes in one process corrupt the heap. "
            "Do not import torch (or anything bundling its own HIP runtime) in a process that uses libmgicp.so.")


def load() -> ctypes.CDLL:
    """Load the in-tree libmgicp.so; raise loudly when it is absent (no fallback path) or when a
    second HIP runtime is (or would become) mapped next to it."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build the HIP engine first (python -c 'import __graft_entry__ as g; g.build()' "
            "or `make`). There is no CPU fallback.")
    check_single_hip_runtime("before loading libmgicp.so")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    check_single_hip_runtime("after loading libmgicp.so")
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def default_params() -> MgicpParams:
    p = MgicpParams()
    load().mgicp_default_params(ctypes.byref(p))
    return p
