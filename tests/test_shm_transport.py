"""The node-wide transport of the per-pass sums (csrc/shm_rows.hpp), on the CPU.

libmgicp.so's multi-GPU form without a collective per pass: every rank's GPU writes its super
partials as stamped rows into ONE POSIX shared-memory segment at their global super index, every
rank's host waits for all rows and takes the same fixed-order total.  tests/shm_harness.cpp plays
the GPUs (it writes rows exactly as fdf_server_kernel's finishing waves do) and calls the engine's
own header for everything else, so these tests run the engine's protocol code, in separate processes:
  * attach: creator / joiner race, the all-ranks barrier, the name unlinked afterwards, geometry
    mismatches refused;
  * 40 passes with random delays between ranks (parity-buffer reuse under skew): every rank's total
    equals the fixed-order total of the single-GPU supers, bit for bit, for world 1, 2, 3 and 5;
  * generic gathers (16 and 80 values per super: fitness, GN moments) likewise.
"""
import ctypes
import multiprocessing as mp
import os
import random
import subprocess

import numpy as np
import pytest

from leica_point_cloud_processing_amd.parallel import super_first

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("shm") / "libshm_harness.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-shared", "-fPIC", "-o", out,
                    os.path.join(HERE, "shm_harness.cpp"), "-lrt"], check=True)
    return out


def _load(path):
    lib = ctypes.CDLL(path)
    D = ctypes.POINTER(ctypes.c_double)
    lib.h_attach.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_double]
    lib.h_error.restype = ctypes.c_char_p
    lib.h_write_rows.argtypes = [ctypes.c_uint, ctypes.c_longlong, ctypes.c_longlong, D]
    lib.h_wait_total.argtypes = [ctypes.c_uint, ctypes.c_longlong, D, ctypes.c_double]
    lib.h_gather.argtypes = [ctypes.c_ulonglong, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong,
                             ctypes.c_int, D, D, ctypes.c_double]
    return lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def fixed_total(rows: np.ndarray) -> np.ndarray:
    """wave_total's order (mgicp_kernels.hip), host mirror in parallel.py."""
    from leica_point_cloud_processing_amd.parallel import fixed_total as ft

    return ft(list(rows))


def _table(seed, npass, nsup, nv):
    rng = np.random.default_rng(seed)
    # magnitudes spread over many binades, so the summation order matters for the last bits
    return rng.standard_normal((npass, nsup, nv)) * np.exp(rng.uniform(-20, 20, (npass, nsup, nv)))


def _rank(path, name, world, rank, nsup, npass, max_sup, q):
    try:
        lib = _load(path)
        if lib.h_attach(name.encode(), world, rank, max_sup, 60.0) != 0:
            q.put((rank, "attach: " + lib.h_error().decode()))
            return
        a, b = super_first(rank, nsup, world), super_first(rank + 1, nsup, world)
        rnd = random.Random(rank)
        rows = _table(7, npass, nsup, 16)
        got = []
        for p in range(npass):
            stamp = p + 1
            if rnd.random() < 0.3:
                import time
                time.sleep(rnd.uniform(0, 0.004))  # skew between ranks
            mine = np.ascontiguousarray(rows[p, a:b])
            lib.h_write_rows(stamp, a, b - a, _dp(mine))
            out = np.zeros(16)
            if lib.h_wait_total(stamp, nsup, _dp(out), 60.0) != 0:
                q.put((rank, f"pass {p}: rows missing"))
                return
            got.append(out)
        gath = []
        for g, nv in enumerate([16, 80, 16, 80, 80]):
            tab = _table(100 + g, 1, nsup, nv)[0]
            mine = np.ascontiguousarray(tab[a:b])
            out = np.zeros(nv)
            if lib.h_gather(g + 1, a, b - a, nsup, nv, _dp(mine), _dp(out), 60.0) != 0:
                q.put((rank, f"gather {g}: flags missing"))
                return
            gath.append(out)
        lib.h_detach()
        q.put((rank, (np.stack(got), gath)))
    except Exception as exc:  # noqa: BLE001 -- report to the parent
        q.put((rank, repr(exc)))


@pytest.mark.parametrize("world,nsup", [(1, 3), (2, 5), (3, 7), (5, 70)])
def test_rows_and_gathers_bitwise_single_gpu_order(harness, world, nsup):
    name = f"/mgicp_test_{os.getpid()}_{world}_{nsup}"
    npass = 40
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(harness, name, world, r, nsup, npass, 128, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    rows = _table(7, npass, nsup, 16)
    want = np.stack([fixed_total(rows[p]) for p in range(npass)])
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
        got, gath = res[r]
        np.testing.assert_array_equal(got, want)  # bitwise: the single-GPU tree
        for g, nv in enumerate([16, 80, 16, 80, 80]):
            np.testing.assert_array_equal(gath[g], fixed_total(_table(100 + g, 1, nsup, nv)[0]))
    assert not os.path.exists("/dev/shm" + name)  # unlinked once every rank had mapped it


def _attach_only(path, name, world, rank, max_sup, q):
    lib = _load(path)
    rc = lib.h_attach(name.encode(), world, rank, max_sup, 3.0)
    q.put((rank, rc, lib.h_error().decode()))


def test_attach_refuses_mismatched_geometry_and_times_out(harness):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/mgicp_test_geom_{os.getpid()}"
    procs = [ctx.Process(target=_attach_only, args=(harness, name, 2, r, 64 if r == 0 else 65, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    assert any(rc != 0 and "geometry" in err for _, rc, err in res), res
    # a lone rank of a world of 2 gives up at its timeout (3 s) instead of hanging
    name2 = f"/mgicp_test_lone_{os.getpid()}"
    lib = _load(harness)
    assert lib.h_attach(name2.encode(), 2, 0, 8, 1.0) != 0
    assert "timed out" in lib.h_error().decode()
    for n in (name, name2):
        try:
            os.unlink("/dev/shm" + n)
        except FileNotFoundError:
            pass


def test_fixed_total_matches_device_order_definition():
    """The host total is the device's wave_total order, not a plain sequential sum: for a table
    whose magnitudes make the order visible the two differ, and fixed_total agrees with a direct
    transcription of the shuffle tree (lane i takes lane i + off for off = 32 .. 1)."""
    rows = _table(3, 1, 200, 4)[0]
    seq = np.zeros(4)
    for s in range(200):
        seq = seq + rows[s]
    ft = fixed_total(rows)
    assert not np.array_equal(ft, seq)
    lanes = np.zeros((64, 4))
    for l in range(64):
        for s in range(l, 200, 64):
            lanes[l] = lanes[l] + rows[s]
    v = lanes.copy()
    for off in (32, 16, 8, 4, 2, 1):
        v = np.array([v[i] + v[i + off] if i + off < 64 else v[i] + v[i] for i in range(64)])
    np.testing.assert_array_equal(ft, v[0])
