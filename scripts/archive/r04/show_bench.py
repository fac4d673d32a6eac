"""one-line summary of a bench.py JSON line (GPU job logs)"""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
k = d["kernels"]
print(d["config"]["name"], "value", d["value"], "ms/step", d["ms_per_step"], "its", d["iterations_per_align"],
      "passes", d["objective_passes_per_align"], "| frac", r["frac"], "us/pass", round(r["avg_launch_ms"] * 1e3, 2),
      "timing-form frac", (r.get("timing_form") or {}).get("frac_52B"),
      "| corr ms", round(k["correspond"]["avg_ms"], 4), "compact ms", round(k["compact_mahalanobis"]["avg_ms"], 4),
      "knn ms", round(k["knn_cov"]["avg_ms"], 4),
      "| parity", (d.get("parity_full_size") or {}).get("frob_vs_oracle"),
      "| new clouds", d.get("ms_to_converge_new_clouds_warm_process"),
      "| stats", d.get("pass_stats_timed"), "| ncorr", d.get("n_corr"))
