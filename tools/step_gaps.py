"""Per-step timeline from tools/step_trace.sh output: screen/verify durations and the gaps between screens."""
import csv, glob, statistics, sys
d = sys.argv[1]
ks = []
for f in glob.glob(f"{d}/t/**/*kernel_trace.csv", recursive=True):
    ks += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
ks.sort()
scr = [(a, b) for a, b, n in ks if "sk_score_kernel<" in n and n.split("sk_score_kernel<")[1].split(">")[0].split(",")[6].strip() == "0"]
ver = [(a, b) for a, b, n in ks if "sk_score_kernel<" in n and n.split("sk_score_kernel<")[1].split(">")[0].split(",")[6].strip() == "1"]
other = [(a, b, n[:50]) for a, b, n in ks if "sk_score_kernel" not in n]
tail = scr[-150:]
dur = [(b - a) / 1e3 for a, b in tail]
gap = [(tail[i + 1][0] - tail[i][1]) / 1e3 for i in range(len(tail) - 1)]
per = [(tail[i + 1][0] - tail[i][0]) / 1e3 for i in range(len(tail) - 1)]
print("screens", len(scr), "verifies", len(ver), "others", len(other))
print("screen us median", statistics.median(dur), "gap median", statistics.median(gap), "start-to-start median", statistics.median(per))
vd = [(b - a) / 1e3 for a, b in ver[-150:]]
print("verify us median", statistics.median(vd) if vd else None)
# overlap of verify with screens
print("sample timeline (us, rel):")
t0 = tail[-6][0]
ev = sorted([(a, b, "S") for a, b in tail[-6:]] + [(a, b, "V") for a, b in ver if a >= t0 - 100000][-6:])
for a, b, n in ev:
    print(f"  {n} {(a - t0) / 1e3:8.1f} .. {(b - t0) / 1e3:8.1f}")
cps = []
for f in glob.glob(f"{d}/t/**/*memory_copy_trace.csv", recursive=True):
    cps += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "")) for r in csv.DictReader(open(f))]
print("memory copies", len(cps))
