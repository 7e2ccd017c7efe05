"""Host-side enqueue cost of one search step (no device sync inside the loop), next to the device step
time, for one shard and for two shards on one device (the pipelined-exchange path with peer copies).
If the enqueue cost approached the device step time, small shards (N = 8: 125k rows) would be host-bound.
usage: python tools/host_enqueue.py [rows] [steps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rag-serving-system_amd"))
from rag_service_amd import Index  # noqa: E402
from rag_service_amd import _lib  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
q = np.random.default_rng(5).standard_normal((32, 1024)).astype(np.float32)
for devs in ([0], [0, 0]):
    ix = Index(devices=devs, dtype="fp32", metric="cosine")
    ix.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, rows * len(devs), 1024)
    ix.set_queries(q)
    for _ in range(20):
        ix.search_staged(5)
    ix.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ix.search_staged(5)
    t1 = time.perf_counter()
    ix.synchronize()
    t2 = time.perf_counter()
    print({"shards": len(devs), "rows_per_shard": rows, "host_enqueue_us_per_step": round((t1 - t0) / steps * 1e6, 2),
           "device_us_per_step": round((t2 - t0) / steps * 1e6, 2)}, flush=True)
    ix.close()
