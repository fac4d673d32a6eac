#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs into per-launch HBM bytes of the path's kernels.

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports exactly HALF of the bytes of a wide (16 B/lane) coalesced
STREAMING read, and "other access widths are uncalibrated".  So the x2 correction is applied per
kernel only where the kernel's reads are all 16-byte-per-lane coalesced streams:
  * fdf_soa_kernel and the resident server's streamed part (fdf_server_kernel<true, W>) -- every load
    is a float4 / double2 stream at consecutive addresses: x2;
  * correspond_kernel, the 1-NN cell-list kernels, knn_cov_kernel, fitness / segdiff (grid gathers),
    the compaction kernels and gn_moments_kernel (coalesced 4 B index loads mixed with 16 B gathers): raw FETCH_SIZE,
    labelled uncalibrated -- the true HBM bytes lie between 1x and 2x the raw figure.
WRITE_SIZE is taken as is.  FETCH_SIZE and WRITE_SIZE come from separate --pmc passes.

usage: pmc_summary.py FETCH_DIR WRITE_DIR N_SOURCE WORLD OUT_JSON
"""
import csv
import glob
import json
import os
import sys

STREAMING = {"fdf_soa_kernel", "fdf_server_kernel<true"}
# the resident pass server's timing form (fdf_server_kernel<true, W>) runs PASSES passes per dispatch (bench.py
# --pass-bench-passes): its figures are per pass (dispatch / PASSES, the one-time resident load
# included pro rata)
PASSES = {"fdf_server_kernel<true": int(os.environ.get("PASS_BENCH_PASSES", "50"))}
KERNELS = ("fdf_server_kernel<true", "fdf_soa_kernel", "vl_query_compact_kernel", "vl_query_kernel",
           "vl_fallback_kernel", "vl_build_kernel", "chunk_compact_list_kernel", "chunk_compact_kernel",
           "correspond_wave_kernel", "correspond_kernel", "knn_cov2_kernel",
           "knn_cov_kernel", "fitness_kernel", "gn_moments_kernel", "segdiff_kernel", "voxel_key_kernel",
           "voxel_centroid_kernel")


def per_dispatch(directory, counter, kernel):
    vals = []
    for path in glob.glob(os.path.join(directory, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == counter and kernel in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return vals


# r04: the listed sweep's kernels run in three states in one bench run (the align that builds the
# lists defers most chunks to the compaction launch; the timed aligns defer none): their figure is the
# MEDIAN dispatch, i.e. the steady state the timed aligns run
MEDIAN = {"vl_query_compact_kernel", "chunk_compact_list_kernel"}


def entry(fk, wk, streaming, passes=1, median=False):
    if median:
        f_kib = sorted(fk)[len(fk) // 2] / passes
        w_kib = sorted(wk)[len(wk) // 2] / passes
    else:
        f_kib = sum(fk) / len(fk) / passes
        w_kib = sum(wk) / len(wk) / passes
    mult = 2.0 if streaming else 1.0
    return {
        "dispatches": len(fk),
        "fetch_size_kib_raw_avg": f_kib,
        "write_size_kib_raw_avg": w_kib,
        "hbm_bytes_per_launch": mult * f_kib * 1024 + w_kib * 1024,
        "correction": ("2 x FETCH_SIZE x 1024 (gfx950 wide streaming read halving) + WRITE_SIZE x 1024"
                       if streaming else
                       "raw FETCH_SIZE x 1024 + WRITE_SIZE x 1024; gather / mixed access widths are "
                       "uncalibrated on gfx950: true HBM bytes between 1x and 2x the raw fetch"),
    }


def main():
    fdir, wdir, n_source, world, out = sys.argv[1:6]
    kernels = {}
    for k in KERNELS:
        fk, wk = per_dispatch(fdir, "FETCH_SIZE", k), per_dispatch(wdir, "WRITE_SIZE", k)
        if fk and wk:
            kernels[k] = entry(fk, wk, k in STREAMING, PASSES.get(k, 1), k in MEDIAN)
            if k in MEDIAN:
                kernels[k]["per"] = "median dispatch (steady state of the timed aligns)"
            if k in PASSES:
                kernels[k]["per"] = f"pass (dispatch / {PASSES[k]})"
    if "fdf_server_kernel<true" in kernels:  # bench.py's key for the server's roofline traffic
        kernels["fdf_server_kernel"] = kernels.pop("fdf_server_kernel<true")
    # the sweep + compaction of the timed aligns: r04 the fused listed sweep (vl_query_compact_kernel,
    # its deferred chunks in chunk_compact_list_kernel), before the r03 sweep + its compaction
    if "vl_query_compact_kernel" in kernels:
        parts = [kernels["vl_query_compact_kernel"]] + [kernels[k] for k in ("chunk_compact_list_kernel",) if k in kernels]
    else:
        sweep = "correspond_wave_kernel" if "correspond_wave_kernel" in kernels else "correspond_kernel"
        comp = "chunk_compact_kernel"
        parts = [kernels[k] for k in (sweep, comp) if k in kernels] if sweep in kernels and comp in kernels else []
    if parts:
        kernels["correspond_plus_compact"] = {
            "hbm_bytes_per_launch": sum(p["hbm_bytes_per_launch"] for p in parts),
            "correction": parts[0]["correction"],
        }
    if "fdf_soa_kernel" not in kernels:
        raise SystemExit("no counters found for fdf_soa_kernel")
    res = {"n_source": int(n_source), "world": int(world), "kernels": kernels,
           "fdf_hbm_bytes_per_launch": kernels["fdf_soa_kernel"]["hbm_bytes_per_launch"]}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
