"""Median per-launch SQ counters of the similarity kernel from tools/ab/sq_passes.sh output dirs."""
import csv, glob, statistics, sys, collections
for d in sys.argv[1:]:
    per = collections.defaultdict(list)
    for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "sk_score_kernel" in r["Kernel_Name"] or "fused_score_kernel" in r["Kernel_Name"]:
                per[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d, {k: f"{statistics.median(v):.4g}" for k, v in sorted(per.items())})
