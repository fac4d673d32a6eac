"""r06: the 1-NN cell lists' build cost at C4.  Two patterns on one engine each:
(a) the default policy -- aligns 1..6 after set_source / set_target (lists built by aligns 3-4);
(b) every queried cell built in the first align (debug options vlist_cold 0, vlist_eager 1): the
all-cells build, then two aligns on the built lists.
usage: [MGICP_LIB_NAME=...] python3 scripts/r06/vlb_time.py [C4F]"""
import os, sys, time, json
sys.path.insert(0, os.getcwd())
from leica_point_cloud_processing_amd import synth
from leica_point_cloud_processing_amd.engine import GICPEngine

c4f = len(sys.argv) > 1 and sys.argv[1] == "C4F"
scan, cad, _ = synth.scan_vs_cad(5_000_000, 5_000_000, clutter=0.04 if c4f else 0.0, debris=40_000 if c4f else 0)
lib = os.environ.get("MGICP_LIB_NAME", "libmgicp.so")
res = {"lib": lib, "config": "C4F" if c4f else "C4"}
for name, opts, n in (("default", {"target_cache": 0}, 6),
                      ("eager_all", {"vlist_cold": 0, "vlist_eager": 1, "target_cache": 0}, 3)):
    e = GICPEngine(options=opts)
    e.set_source_xyz(scan)
    e.set_target_xyz(cad)
    rows = []
    for a in range(n):
        t0 = time.perf_counter()
        e.align()
        wall = 1e3 * (time.perf_counter() - t0)
        st = e.vlist_stats()
        T = e.getFinalTransformation() if hasattr(e, "getFinalTransformation") else None
        rows.append({"align": a + 1, "ms_wall": round(wall, 2), "ms_loop": round(e.last_result["ms_loop"], 2),
                     "its": e.last_result["iterations"], "lists": st.get("lists"), "entries": st.get("entries"),
                     "overflow": st.get("overflow"), "reject": st.get("reject"),
                     "T": None if T is None else [float(x) for x in list(T.ravel())]})
        print(name, json.dumps({k: v for k, v in rows[-1].items() if k != "T"}), flush=True)
    res[name] = rows
    e.close()
# every align of a pattern must end on the same transform (lists change no result)
for name in ("default", "eager_all"):
    Ts = [r["T"] for r in res[name]]
    res[name + "_same_T"] = all(t == Ts[0] for t in Ts)
res["cross_same_T"] = res["default"][0]["T"] == res["eager_all"][0]["T"]
print("SUMMARY", json.dumps({k: v for k, v in res.items() if not isinstance(v, list)}), flush=True)
