#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs into per-launch HBM bytes of one kernel.

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md "HBM" (and cdna_hip_programming.md
section 7): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half of
the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled here -- the objective
pass reads only 16-byte-per-lane vectors (float4, double2).  WRITE_SIZE is taken as is.
FETCH_SIZE and WRITE_SIZE were collected in separate --pmc passes (slot limits).

usage: pmc_summary.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR N_SOURCE WORLD OUT_JSON
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(directory, counter, kernel):
    vals = []
    for path in glob.glob(os.path.join(directory, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == counter and kernel in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, kernel, n_source, world, out = sys.argv[1:7]
    fetch = per_dispatch(fdir, "FETCH_SIZE", kernel)
    write = per_dispatch(wdir, "WRITE_SIZE", kernel)
    if not fetch or not write:
        raise SystemExit(f"no counters found for {kernel}: fetch={len(fetch)} write={len(write)}")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    hbm = 2.0 * f_kib * 1024 + w_kib * 1024
    res = {
        "kernel": kernel,
        "n_source": int(n_source),
        "world": int(world),
        "dispatches_fetch": len(fetch),
        "dispatches_write": len(write),
        "fetch_size_kib_raw_avg": f_kib,
        "write_size_kib_raw_avg": w_kib,
        "fdf_hbm_bytes_per_launch": hbm,
        "correction": "bytes = 2*FETCH_SIZE*1024 (gfx950 wide-read halving) + WRITE_SIZE*1024",
    }
    # the other kernels of the path, for DESIGN.md (same correction; gathers use 16 B/lane loads)
    others = {}
    for k in ("correspond_kernel", "compact_kernel", "knn_cov_kernel", "xform_points", "fitness_kernel",
              "gn_moments_kernel", "segdiff_kernel", "voxel_key_kernel", "voxel_centroid_kernel"):
        fk, wk = per_dispatch(fdir, "FETCH_SIZE", k), per_dispatch(wdir, "WRITE_SIZE", k)
        if fk and wk:
            others[k] = {"dispatches": len(fk),
                         "hbm_bytes_per_launch": 2.0 * sum(fk) / len(fk) * 1024 + sum(wk) / len(wk) * 1024}
    res["other_kernels"] = others
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
