"""Per-call host time of rr_search_staged at the 8-GPU shard size (125k rows), after a full sync: the first calls of a
burst show the pure enqueue cost (nothing to wait for), later ones any blocking once the runtime's queues fill.
usage: python tools/host_calls.py [rows] [--x]   (--x: 1-rank RCCL communicator, the multi-GPU data path)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rag-serving-system_amd"))
from rag_service_amd import Index, get_unique_id, _lib  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 125_000
ix = Index(dtype="fp32", metric="cosine")
if "--x" in sys.argv:
    ix.init_dist(1, 0, get_unique_id())
ix.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, rows, 1024)
q = np.random.default_rng(5).standard_normal((32, 1024)).astype(np.float32)
ix.set_queries(q)
for _ in range(50):
    ix.search_staged(5)
ix.synchronize()
for burst in range(3):
    ix.synchronize()
    ts = []
    t0 = time.perf_counter()
    for _ in range(60):
        a = time.perf_counter()
        ix.search_staged(5)
        ts.append((time.perf_counter() - a) * 1e6)
    t_enq = time.perf_counter() - t0
    ix.synchronize()
    t_all = time.perf_counter() - t0
    print({"burst": burst, "first10_us": [round(x, 1) for x in ts[:10]], "median_first20_us": round(float(np.median(ts[:20])), 1),
           "median_last20_us": round(float(np.median(ts[-20:])), 1), "enqueue_us_per_step": round(t_enq / 60 * 1e6, 1),
           "device_us_per_step": round(t_all / 60 * 1e6, 1)})
# the pure cost of a trivial C-ABI call (ctypes + library entry), for scale
a = time.perf_counter()
for _ in range(1000):
    ix.compute_streams()
print({"ctypes_call_us": round((time.perf_counter() - a) / 1000 * 1e6, 2)})
ix.close()
