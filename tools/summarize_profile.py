"""Summarise rocprofv3 output dirs into one JSON: per-kernel stats (kernel-trace pass) and the fused
kernel's HBM traffic (FETCH_SIZE pass; KiB, x2 on gfx950 per MI355X_MICROARCH.md §HBM).
usage: python tools/summarize_profile.py <stats_dir> <pmc_dir> <alg_bytes_per_launch> > out.json"""
import csv
import glob
import json
import os
import statistics
import sys

stats_dir, pmc_dir, alg = sys.argv[1], sys.argv[2], float(sys.argv[3])
out = {"kernels": [], "fused_traffic": None}
for f in glob.glob(os.path.join(stats_dir, "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        out["kernels"].append({"name": r["Name"], "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                               "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
                               "pct": float(r["Percentage"])})
vals = []
for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if ("sk_score_kernel" in r["Kernel_Name"] or "fused_score_kernel" in r["Kernel_Name"]) \
                and r["Counter_Name"] == "FETCH_SIZE":
            vals.append(float(r["Counter_Value"]))
if vals:
    b = statistics.median(vals) * 1024 * 2
    out["fused_traffic"] = {"launches": len(vals), "fetch_size_kib_median": statistics.median(vals),
                            "hbm_bytes_per_launch": b, "alg_bytes_per_launch": alg, "traffic_over_alg": b / alg}
json.dump(out, sys.stdout, indent=1)
print()
