"""Summarise a tools/profile.sh run into profiles/<tag>/ (kernel stats + PMC per dispatch).

Traffic per launch follows MI355X_MICROARCH.md §HBM for gfx950: FETCH_SIZE and WRITE_SIZE
are in KiB; FETCH_SIZE reports half the bytes of a wide coalesced read, so it is doubled
before comparing with a byte count; WRITE_SIZE is exact for 16-byte-per-lane stores (the
obs stores).  Usage: python tools/summarize_profile.py gpurun_out/prof_<tag> profiles/<tag>
"""
import csv
import re
import json
import os
import shutil
import sys


def kernel_rows(path, kernel):
    rows = list(csv.DictReader(open(path)))
    return [r for r in rows if re.search(kernel, r["Kernel_Name"])]


def main(src, dst, kernel=r"wab_kernel<0|wab_step_q4"):
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    for log in ("bench_trace.log",):
        if os.path.exists(os.path.join(src, log)):
            shutil.copy(os.path.join(src, log), os.path.join(dst, log))
    summ = {"kernel": kernel}
    for r in csv.DictReader(open(stats)):
        if re.search(kernel, r["Name"]):
            summ["trace"] = {"name": r["Name"], "calls": int(r["Calls"]),
                             "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                             "max_ns": float(r["MaxNs"])}
    pmc = {}
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if sub.startswith("pmc") and os.path.exists(f):
            for r in kernel_rows(f, kernel):
                pmc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    summ["pmc_mean_per_dispatch"] = {k: sum(v) / len(v) for k, v in pmc.items()}
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        f = summ["pmc_mean_per_dispatch"]["FETCH_SIZE"] * 1024.0
        w = summ["pmc_mean_per_dispatch"]["WRITE_SIZE"] * 1024.0
        summ["hbm_bytes_per_launch"] = {"fetch_raw": f, "fetch_corrected_x2": 2 * f, "write": w,
                                        "total_corrected": 2 * f + w}
    json.dump(summ, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
