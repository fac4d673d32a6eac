"""r05: where the 1-NN cell lists' build time goes (MGICP_VL_DIAG builds): C4, lists from the first sweep,
every queried cell built at once (debug options vlist_cold 0, vlist_eager 1); the per-sweep [vl-build]
lines on stderr, the align times on stdout.
usage: MGICP_LIB_NAME=libmgicp_vld.so python3 scripts/r05/vl_build_diag.py"""
import os, sys, time
sys.path.insert(0, os.getcwd())
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

scan, cad, _ = synth.scan_vs_cad(5_000_000, 5_000_000)
e = GICPEngine(options={"vlist_cold": 0, "vlist_eager": int(sys.argv[1]) if len(sys.argv) > 1 else 1,
                        "target_cache": 0})
e.set_source_xyz(scan)
e.set_target_xyz(cad)
for a in range(3):
    t0 = time.perf_counter()
    e.align()
    print(f"align {a + 1}: {1e3 * (time.perf_counter() - t0):.2f} ms, loop {e.last_result['ms_loop']:.2f} ms",
          e.vlist_stats(), flush=True)
    sys.stderr.flush()
e.close()
