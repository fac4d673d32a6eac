"""one-screen summary of a bench.py JSON line"""
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms/step", d["ms_per_step"], "frob", d["frob_vs_oracle"], "frac", d["roofline"]["frac"],
      "pass_ms", d["roofline"]["avg_launch_ms"])
cp = d.get("cold_pair") or {}
print("cold_pair", json.dumps({k: v for k, v in cp.items() if k not in ("repeats", "pattern")}))
g = d.get("gicpstate_cycles") or {}
print("gicpstate", json.dumps({k: v for k, v in g.items() if k not in ("cycles", "pattern")}),
      [(c["target_adopted"], c["ms_set_clouds"], c["align"][0]["ms_loop"], c["align"][1]["ms_loop"]) for c in g.get("cycles", [])])
print("new_clouds", json.dumps(d["ms_to_converge_new_clouds_warm_process"]))
r = d["rooflines"]
c5 = r.get("fdf_52B_c5_past_infinity_cache") or {}
print("c5 pass", c5.get("avg_launch_ms"), "frac", c5.get("frac"))
print("knn", r["knn_cov"]["avg_launch_ms"], r["knn_cov"]["frac"], "corr", r["correspondence_plus_mahalanobis"]["avg_launch_ms"])
print("cpu", (d.get("cpu_baseline") or {}).get("value"), "ms_first", d["ms_to_converge_first"])
