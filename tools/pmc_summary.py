#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory: per-kernel average of each
PMC counter, plus HBM bytes per launch with the gfx950 corrections of
MI355X_MICROARCH.md §HBM (FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE
reads half the bytes of a wide coalesced stream, so it is reported both raw
and doubled), and the L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS).

usage: pmc_summary.py gpurun_out/prof_<tag> [> profiles/rNN/<tag>_pmc_summary.txt]
"""
import collections
import csv
import glob
import json
import os
import sys


def main(d):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    kernels = sorted({k for k, _ in agg})
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    dur = {}
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            dur[r["Name"]] = float(r["AverageNs"])
    summary = {}
    for k in kernels:
        if k.startswith("__amd"):
            continue
        c = {n: sum(v) / len(v) for (kk, n), v in agg.items() if kk == k}
        summary[k] = {"avg_ns": dur.get(k), "counters": c,
                      "hbm_read_bytes": 2 * c["FETCH_SIZE"] * 1024 if "FETCH_SIZE" in c else None,
                      "hbm_write_bytes": c["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in c else None}
        print(f"kernel: {k}")
        if k in dur:
            print(f"  avg duration          {dur[k] / 1e3:12.1f} us   (kernel trace)")
        for n in sorted(c):
            print(f"  {n:22s}{c[n]:16.1f}")
        fetch = c.get("FETCH_SIZE", 0.0) * 1024
        write = c.get("WRITE_SIZE", 0.0) * 1024
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            print(f"  HBM read  (FETCH_SIZE)      {fetch / 1e6:10.2f} MB/launch raw, "
                  f"{2 * fetch / 1e6:10.2f} MB doubled (gfx950 wide-read correction)")
            print(f"  HBM write (WRITE_SIZE)      {write / 1e6:10.2f} MB/launch")
            if k in dur:
                t = dur[k] * 1e-9
                print(f"  HBM traffic rate            {(fetch + write) / t / 1e9:10.1f} GB/s raw, "
                      f"{(2 * fetch + write) / t / 1e9:10.1f} GB/s corrected")
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
            print(f"  L2 hit rate                 {c['TCC_HIT_sum'] / tot:10.3f}")
        if "GRBM_GUI_ACTIVE" in c and k in dur:
            print(f"  effective clock             {c['GRBM_GUI_ACTIVE'] / 8 / (dur[k] * 1e-9) / 1e9:10.2f} GHz")
        print()
    with open(os.path.join(d, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
