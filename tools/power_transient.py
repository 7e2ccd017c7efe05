"""Per-launch behaviour of the similarity kernel from an idle GPU (development probe, not product).

Runs bursts of back-to-back searches separated by idle gaps, one burst per corpus dtype, so a
rocprofv3 --kernel-trace of this script shows how launch durations evolve after the GPU leaves idle:

    rocprofv3 --kernel-trace -d OUT -o t --output-format csv -- python3 tools/power_transient.py
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rag-serving-system_amd"))

from rag_service_amd import Index, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--idle", type=float, default=3.0)
    ap.add_argument("--dtypes", default="fp32,fp32,fp32-split,bf16")
    args = ap.parse_args()
    rng = np.random.default_rng(5678)
    q = rng.standard_normal((32, 1024)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    cache = {}
    for dt in args.dtypes.split(","):
        if dt not in cache:
            ix = Index(devices=[0], dtype=dt, metric="cosine")
            ix.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, args.docs, 1024)
            ix.set_queries(q)
            cache[dt] = ix
        ix = cache[dt]
        ix.synchronize()
        time.sleep(args.idle)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ix.search_staged(5)
        ix.synchronize()
        dt_s = time.perf_counter() - t0
        print(f"{dt}: {args.steps} steps {dt_s / args.steps * 1e3:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
