#!/usr/bin/env python3
"""Staged-loop timeline of one shard (run under rocprofv3 --kernel-trace inside gpurun, then analyse here).

    rocprofv3 --kernel-trace --output-format csv -d <dir> -o t -- python3 tools/step_timeline.py run [--docs N] [--x] [--restage]
    python3 tools/step_timeline.py analyse <dir>

`run`: a 1-GPU handle on N synthetic unit-norm rows (optionally with a 1-rank RCCL communicator: --x, the multi-GPU
data path), 32 queries staged once, 50 warm-up + 300 timed rr_search_staged steps, a marker launch (queue probe)
between the phases. `analyse`: over the timed steps only — per kernel family the mean span, the GPU's busy fraction
(union of all kernel spans), per compute stream the chain (prep -> screen -> verify) and the gaps between dependent
launches on it."""
import csv
import glob
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rag-serving-system_amd"))


def run(argv):
    import numpy as np
    from rag_service_amd import Index, get_unique_id, _lib
    docs = int(argv[argv.index("--docs") + 1]) if "--docs" in argv else 125000
    ix = Index(dtype="fp32", metric="cosine")
    if "--x" in argv:
        ix.init_dist(1, 0, get_unique_id())
    ix.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, docs, 1024)
    rng = np.random.default_rng(5)
    q = rng.standard_normal((32, 1024)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    ix.set_queries(q)
    stage = lambda i: None
    if "--restage" in argv:   # a new batch resident in HBM staged every step, as bench.py's timed loop
        import torch
        qs = rng.standard_normal((16, 32, 1024)).astype(np.float32)
        qs /= np.linalg.norm(qs, axis=2, keepdims=True)
        dev = torch.from_numpy(qs).to("cuda:0")
        torch.cuda.synchronize()
        ptrs = [dev[i].data_ptr() for i in range(16)]
        stage = lambda i: ix.set_queries_device(ptrs[i % 16], 32, 1024)
    for i in range(50):
        stage(i)
        ix.search_staged(5)
    ix.synchronize()
    ix.stream_queues()            # marker: queue_probe_kernel launches separate warm-up and timed steps
    ix.synchronize()
    t = time.perf_counter()
    for i in range(300):
        stage(i)
        ix.search_staged(5)
    ix.synchronize()
    el = time.perf_counter() - t
    print({"docs": docs, "exchange": "--x" in argv, "restage": "--restage" in argv, "qps": round(32 * 300 / el, 1), "ms_per_step": round(el / 300 * 1e3, 4)})
    ix.close()


def union(iv):
    busy, cur = 0, None
    for a, b in sorted(iv):
        if cur and a <= cur[1]:
            cur[1] = max(cur[1], b)
        else:
            if cur:
                busy += cur[1] - cur[0]
            cur = [a, b]
    return busy + (cur[1] - cur[0] if cur else 0)


def family(n):
    n = n.split("(")[0]
    if "sk_score_kernel<" in n:
        t = n.split("sk_score_kernel<")[1].split(">")[0].split(",")
        return f"sk DT{t[0].strip()} {'verify' if t[6].strip() == '1' else 'screen'}"
    return n.split("<")[0].split("::")[-1]


def analyse(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"]), int(r["Stream_Id"]))
                 for r in csv.DictReader(open(f))]
    rows.sort()
    probes = [r for r in rows if r[2] == "queue_probe_kernel"]
    t0 = probes[-1][1]                                  # after the last marker: the timed steps
    win = [r for r in rows if r[0] >= t0]
    t1 = max(b for _, b, _, _ in win)
    span = (t1 - t0) / 1e3
    print(f"timed window {span:.1f} us, {len([r for r in win if r[2].endswith('screen')])} screens")
    print(f"GPU busy (union of all kernels) {union([(a, b) for a, b, _, _ in win]) / 1e3 / span:.3f} of the window")
    fams = {}
    for a, b, f, s in win:
        fams.setdefault(f, []).append((b - a) / 1e3)
    for f, v in sorted(fams.items(), key=lambda x: -sum(x[1])):
        print(f"  {f:28s} n={len(v):4d} mean {statistics.mean(v):7.2f} us  sum/step {sum(v) / 300:7.2f} us")
    scr = [r for r in win if r[2].endswith("screen")]
    if len(scr) > 2:
        st = [(scr[i + 1][0] - scr[i][0]) / 1e3 for i in range(len(scr) - 1)]
        print(f"screen start-to-start median {statistics.median(st):.2f} us, mean {statistics.mean(st):.2f} us")
    for s in sorted({s for *_, s in win}):
        ks = [r for r in win if r[3] == s]
        if len(ks) < 50:
            continue
        gaps = [(ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
        print(f"stream {s}: {len(ks)} kernels, busy {union([(a, b) for a, b, _, _ in ks]) / 1e3 / span:.3f}, "
              f"gap between consecutive launches median {statistics.median(gaps):.2f} us, mean {statistics.mean(gaps):.2f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2:])
    else:
        analyse(sys.argv[2])
