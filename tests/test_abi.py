"""CPU tests of the drop-in boundary: libmgicp.so loads, exports every symbol the C-ABI header
declares, its ctypes mirrors match the header's structs, and nothing silently falls back to
CPU compute when no GPU is present."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mi355x_gicp.h")


def _struct_fields(name):
    text = open(HEADER).read()
    m = re.search(r"typedef struct \{([^{}]*)\}\s*" + name + ";", text, re.S)
    assert m, name
    body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        typ, names = decl.split(None, 1)
        fields += [(n.strip(), typ) for n in names.split(",")]
    return fields


def test_library_exports_every_header_symbol():
    from leica_point_cloud_processing_amd import _lib

    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib._SIGNATURES), "ctypes signature table out of sync with the header"


@pytest.mark.parametrize("cname,pyname", [("mgicp_params", "MgicpParams"), ("mgicp_result", "MgicpResult")])
def test_struct_layout_matches_header(cname, pyname):
    from leica_point_cloud_processing_amd import _lib

    cls = getattr(_lib, pyname)
    hdr = _struct_fields(cname)
    py = [(n, t) for n, t in cls._fields_]
    assert [n for n, _ in hdr] == [n for n, _ in py]
    cmap = {"int": ctypes.c_int, "double": ctypes.c_double}
    for (n, ct), (_, pt) in zip(hdr, py):
        assert cmap[ct] == pt, n


def test_header_is_plain_c():
    text = open(HEADER).read()
    assert 'extern "C"' in text
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)  # declarations only, not the docs
    for banned in ("torch", "hipStream_t", "Eigen", "pcl::", "std::", "#include <hip"):
        assert banned not in text


def test_default_params_match_reference():
    """GICPAlignment ctor defaults (src/GICPAlignment.cpp:29-32) + PCL GICP defaults."""
    from leica_point_cloud_processing_amd import _lib

    p = _lib.default_params()
    assert (p.max_iter, p.k, p.max_inner_iter) == (100, 20, 20)
    assert (p.tf_eps, p.rot_eps, p.max_corr_dist, p.gicp_eps) == (4e-3, 2e-3, 4e-2, 1e-3)


def test_no_cpu_fallback_without_gpu():
    """On a machine without a GPU the engine refuses to run instead of computing on the CPU."""
    from leica_point_cloud_processing_amd import _lib
    from leica_point_cloud_processing_amd.engine import GICPEngine

    n = ctypes.c_int(0)
    rc = _lib.load().mgicp_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.MgicpError):
        GICPEngine()


def test_product_never_imports_oracle():
    """The oracle is test infrastructure: no product module may reference it."""
    pkg = os.path.join(ROOT, "leica_point_cloud_processing_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert not re.search(r'#include\s*["<][^">]*gicp_ref', text), f
                assert not re.search(r"\bref_[a-z_]+\s*\(", text), f
                assert not re.search(r"^\s*(from oracle|import oracle)", text, re.M), f
                assert "libgicp_ref" not in text, f


@pytest.mark.gpu
def test_cabi_example_plain_cpp_host():
    """adapter/cabi_example (g++, no HIP headers, no torch) drives the C-ABI as the catkin adapter
    does: PCL-mode and GN aligns, VoxelGrid and SegmentDifferences on PointXYZRGB records."""
    import subprocess

    exe = os.path.join(ROOT, "adapter", "cabi_example")
    assert os.path.exists(exe), "build it with `make adapter-example`"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "cabi_example: OK" in out.stdout


def test_second_hip_runtime_is_refused():
    """the observed "double free or corruption" with torch's bundled HIP runtime next
    to ROCm's (parallel.py) is now a guard: _lib.load() raises MgicpError when another libamdhip64
    is mapped.  Run in a child process (import torch maps torch/lib/libamdhip64.so)."""
    import subprocess
    import sys

    code = ("import torch, sys; sys.path.insert(0, %r)\n"
            "from leica_point_cloud_processing_amd import _lib\n"
            "try:\n    _lib.load()\nexcept _lib.MgicpError as e:\n    print('REFUSED', e.code)\n"
            "else:\n    print('LOADED')\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert "REFUSED -5" in r.stdout, r.stdout + r.stderr
    # and the plain process (no torch) loads it
    code2 = ("import sys; sys.path.insert(0, %r)\nfrom leica_point_cloud_processing_amd import _lib\n"
             "_lib.load(); print('LOADED', sorted(_lib._mapped_hip_runtimes()))\n") % ROOT
    r2 = subprocess.run([sys.executable, "-c", code2], capture_output=True, text=True, timeout=300)
    assert "LOADED" in r2.stdout and "torch" not in r2.stdout, r2.stdout + r2.stderr


@pytest.mark.parametrize("k", [0, 33, -1])
def test_k_out_of_range_is_invalid(k):
    """k_correspondences outside [1, 32] is refused before any device work (include/mi355x_gicp.h)."""
    from leica_point_cloud_processing_amd import _lib

    lib = _lib.load()
    p = _lib.default_params()
    p.k = k
    h = ctypes.c_void_p()
    assert lib.mgicp_create(ctypes.byref(h), ctypes.byref(p)) == _lib.MGICP_E_INVALID
