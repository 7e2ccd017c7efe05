#!/usr/bin/env python3
"""Hardware-queue placement from a rocprofv3 kernel trace (+ memory-copy trace): per (Queue_Id, Stream_Id), the
kernel families and copy kinds dispatched there, so a reader can see which streams share an in-order hardware queue.

    python tools/queue_map.py <dir with *kernel_trace.csv [*memory_copy_trace.csv]> [--md]
"""
import collections
import csv
import glob
import sys


def family(name: str) -> str:
    n = name.split("(")[0].replace("void ", "")
    if "sk_score_kernel<" in n:
        t = n.split("sk_score_kernel<", 1)[1].split(">", 1)[0].split(",")
        mode = t[6].strip() if len(t) > 6 else "?"
        return f"sk_score_kernel DT {t[0].strip()} MODE {mode}" + (" (verify)" if mode == "1" else "")
    if "rccl" in n.lower() or "nccl" in n.lower():
        return "RCCL " + n.split("<")[0].split("::")[-1]
    return n.split("<")[0].split("::")[-1]


def main():
    d = sys.argv[1]
    md = "--md" in sys.argv
    per = collections.defaultdict(collections.Counter)
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            per[(int(r["Queue_Id"]), int(r["Stream_Id"]))][family(r["Kernel_Name"])] += 1
    for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            q = r.get("Queue_Id")
            st = r.get("Stream_Id")
            if q is None or st is None:
                continue
            per[(int(q), int(st))]["copy " + r.get("Direction", "?")] += 1
    if md:
        print("| Queue_Id | Stream_Id | work (launches) |")
        print("|---|---|---|")
    for (q, st), c in sorted(per.items()):
        work = ", ".join(f"{k} x{v}" for k, v in c.most_common())
        print(f"| {q} | {st} | {work} |" if md else f"queue {q} stream {st}: {work}")


if __name__ == "__main__":
    main()
