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
    m = summ["pmc_mean_per_dispatch"]
    if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVES" in m:
        # SQ_ACTIVE_INST_VALU tracks SQ_INSTS_VALU one for one on this kernel shape, so it is
        # taken as instructions.  A SIMD-32 issues one wave64 VALU instruction per 2 cycles when
        # two or more waves feed it (MI355X_MICROARCH.md: v_fma_f32 2 cyc; 4 for one wave
        # alone), so the pipe's busy fraction counts 2 cycles per instruction (rounds 1-4 of
        # this repo counted 4, twice the pipe's occupancy).  The launch's cycles are its
        # rocprofv3 duration at the nominal 2.4 GHz: GRBM_GUI_ACTIVE / 8 reads high on
        # dispatches this short (MI355X_MICROARCH.md, DVFS give-back).
        simds = 256 * 4
        v = {"insts_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"],
             "salu_insts_per_wave": m.get("SQ_INSTS_SALU", 0.0) / m["SQ_WAVES"],
             "issue_cycles_per_simd": 2.0 * m["SQ_ACTIVE_INST_VALU"] / simds}
        if "trace" in summ:
            cyc = summ["trace"]["avg_ns"] * 2.4
            v["launch_cycles_at_2.4GHz"] = cyc
            v["busy_frac"] = v["issue_cycles_per_simd"] / cyc
        v["source"] = ("SQ_INSTS_VALU / SQ_WAVES; busy = 2 cycles * SQ_ACTIVE_INST_VALU / 1024 SIMDs / "
                       "(rocprofv3 avg duration * 2.4 GHz)")
        summ["valu"] = v
    json.dump(summ, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
