"""r04: where a warm process's new-clouds time goes -- set_target / set_source / align wall times of a
fresh engine after a first one ran (bench.py's ms_to_converge_new_clouds leg), with the engine's
MGICP_TRACE phase stamps on stderr.  usage: MGICP_TRACE=1 python3 scripts/r04/new_clouds_trace.py"""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

scan, cad, T = synth.scan_vs_cad(5_000_000, 5_000_000)
e = GICPEngine(); e.set_target_xyz(cad); e.set_source_xyz(scan); e.align(); e.close()
for rep in range(3):
    e = GICPEngine()
    print(f"---- rep {rep}: new engine ----", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    if os.environ.get("SOURCE_FIRST") == "1":  # the reference's order (GICPAlignment.cpp:89-90)
        e.set_source_xyz(scan)
        t1 = time.perf_counter()
        e.set_target_xyz(cad)
    else:
        e.set_target_xyz(cad)
        t1 = time.perf_counter()
        e.set_source_xyz(scan)
    t2 = time.perf_counter()
    e.align()
    t3 = time.perf_counter()
    r = e.last_result
    print(f"rep {rep} ({'source' if os.environ.get('SOURCE_FIRST') == '1' else 'target'} first): set_* {1e3*(t1-t0):.3f} ms, set_* {1e3*(t2-t1):.3f} ms, align {1e3*(t3-t2):.3f} ms, "
          f"total {1e3*(t3-t0):.3f} ms | upload {r['ms_upload']:.3f} prep {r['ms_prep']:.3f} loop {r['ms_loop']:.3f}",
          flush=True)
    e.close()
