"""Median per-launch SQ counters of the similarity kernels from tools/ab/sq_passes.sh output dirs, per kernel
(template arguments), with per-tile-per-wave instruction rates for the split-K kernel (tiles = rows / 32 given as
--rows; waves = 8 per workgroup)."""
import collections
import csv
import glob
import json
import statistics
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--rows=")]
    rows = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--rows=")), 0)
    out = {}
    for d in args:
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                n = r["Kernel_Name"]
                if "sk_score_kernel" in n or "fused_score_kernel" in n:
                    key = n.split("(")[0].replace("void rr::sk::", "")
                    per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        res = {}
        for k, c in per.items():
            med = {name: statistics.median(v) for name, v in sorted(c.items())}
            if rows and "SQ_INSTS_MFMA" in med and ", 0, " in k:
                tw = rows / 32 * 8
                med["per_tile_wave"] = {n.replace("SQ_INSTS_", ""): round(med[n] / tw, 1)
                                        for n in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                                                  "SQ_INSTS_BRANCH") if n in med}
            res[k] = med
        out[d] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
