"""Where a short timed window's time goes (bench.py timed_steps): per phase of the closing sequence and the window's
fixed part, fitted over K (window(K) = fixed + K x step).
usage: python tools/window_cost.py [rows] [--x]   (--x: 1-rank RCCL communicator, the multi-GPU data path)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rag-serving-system_amd"))
from rag_service_amd import Index, get_unique_id, _lib  # noqa: E402
import torch  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 125_000
torch.cuda.set_device(0)
ix = Index(dtype="fp32", metric="cosine")
if "--x" in sys.argv:
    ix.init_dist(1, 0, get_unique_id())
ix.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, rows, 1024)
q = np.random.default_rng(5).standard_normal((32, 1024)).astype(np.float32)
q /= np.linalg.norm(q, axis=1, keepdims=True)
ix.set_queries(q)
for _ in range(300):
    ix.search_staged(5)
ix.synchronize()


def window(K, warm=5):
    for _ in range(warm):
        ix.search_staged(5)
    ix.synchronize()
    torch.cuda.synchronize()
    ix.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        ix.search_staged(5)
    t1 = time.perf_counter()
    ix.screen_counts_all()
    t2 = time.perf_counter()
    ix.synchronize()
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    return [(t - t0) * 1e6 for t in (t1, t2, t3, t4)]


res = {}
for K in (1, 2, 5, 10, 20, 40, 80):
    runs = np.array([window(K) for _ in range(15)])
    med = np.median(runs, axis=0)
    res[K] = med
    print({"K": K, "enqueue_us": round(med[0], 1), "counts_us": round(med[1], 1), "sync_us": round(med[2], 1),
           "total_us": round(med[3], 1), "us_per_step": round(med[3] / K, 2)}, flush=True)
Ks = np.array(sorted(res))
tot = np.array([res[k][3] for k in Ks])
A = np.vstack([np.ones_like(Ks, dtype=float), Ks.astype(float)]).T
(fixed, step), *_ = np.linalg.lstsq(A, tot, rcond=None)
print({"fit_fixed_us": round(float(fixed), 1), "fit_step_us": round(float(step), 2)})
# idle costs of the closing calls
for name, fn in (("screen_counts_all", ix.screen_counts_all), ("synchronize", ix.synchronize),
                 ("torch_sync", torch.cuda.synchronize)):
    a = time.perf_counter()
    for _ in range(200):
        fn()
    print({"idle_" + name + "_us": round((time.perf_counter() - a) / 200 * 1e6, 2)})
ix.close()
