"""Per-launch device time of a kernel whose launches overlap (two compute streams): the union of its launches'
[start, end) spans in a rocprofv3 kernel trace, divided by the number of launches, next to the mean span.
usage: python tools/trace_union.py <kernel_trace.csv> [kernel-name substring, default 'sk_score_kernel<7']"""
import csv
import json
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "sk_score_kernel<7"
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"])
busy, cur = 0, None
for a, b in iv:
    if cur and a <= cur[1]:
        cur[1] = max(cur[1], b)
    else:
        if cur:
            busy += cur[1] - cur[0]
        cur = [a, b]
if cur:
    busy += cur[1] - cur[0]
n = len(iv)
print(json.dumps({"kernel": pat, "launches": n, "union_us_per_launch": round(busy / max(n, 1) / 1e3, 2),
                  "mean_span_us": round(sum(b - a for a, b in iv) / max(n, 1) / 1e3, 2)}))
