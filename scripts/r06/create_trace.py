"""r06: where mgicp_create's time goes: two engines in one process with the engine's
trace points on (MGICP_TRACE=1, stderr), the wall time of each creation on stdout.
usage: MGICP_TRACE=1 python3 scripts/r06/create_trace.py"""
import os, sys, time, ctypes
sys.path.insert(0, os.getcwd())
t0 = time.perf_counter()
from leica_point_cloud_processing_amd import _lib
lib = _lib.load()
t1 = time.perf_counter()
print(f"load (dlopen libmgicp + HIP + RCCL): {1e3 * (t1 - t0):.2f} ms", flush=True)
n = ctypes.c_int(0)
from leica_point_cloud_processing_amd.engine import GICPEngine
for i in range(2):
    sys.stderr.write(f"[py] engine {i + 1} create begin\n"); sys.stderr.flush()
    ta = time.perf_counter()
    e = GICPEngine()
    tb = time.perf_counter()
    sys.stderr.write(f"[py] engine {i + 1} create end\n"); sys.stderr.flush()
    print(f"engine {i + 1} create: {1e3 * (tb - ta):.2f} ms", flush=True)
    e.close()
