#!/usr/bin/env python3
"""Why a clustered corpus's block still flags (diagnostic; needs tools/ab/librag_retrieval_diag.so, built with
-DRR_VERIFY_DIAG): 1M-row interleaved SQuAD clusters (tools/clustered_bench.py), full lane lists from the start,
synchronous searches; for every flagged block print the failing query slots' [k-th largest bound, largest
single-list bound, phase-1 exact k-th, phase-2 exact k-th, |R|, decision, complete]."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "rag-serving-system_amd"), os.path.join(REPO, "tools")]
os.environ["RR_LIBRARY"] = os.path.join(REPO, "tools", "ab", "librag_retrieval_diag.so")
os.environ["RR_SCREEN_FULL_LISTS"] = "1"
from clustered_bench import build  # noqa: E402
from rag_service_amd import Index, _lib  # noqa: E402


def f(key):
    o = (int(key) >> 32) & 0xFFFFFFFF
    u = (o & 0x7FFFFFFF) if (o & 0x80000000) else (~o & 0xFFFFFFFF)
    return float(np.array([u], np.uint32).view(np.float32)[0]), 0xFFFFFFFF - (int(key) & 0xFFFFFFFF)


def main():
    sigma, layout, n = float(sys.argv[1]) if len(sys.argv) > 1 else 0.01, "interleaved", 1_000_000
    squad = np.load(os.path.join(REPO, "tests", "golden", "data", "squad_embeddings.npy")).astype(np.float32)
    squad /= np.linalg.norm(squad, axis=1, keepdims=True)
    rng = np.random.default_rng(20260)
    noise = rng.standard_normal((n, 1024), dtype=np.float32) / np.float32(32.0)
    qrng = np.random.default_rng(777)
    qc = qrng.integers(0, 1000, 32)
    qnoise = qrng.standard_normal((32, 1024), dtype=np.float32) / np.float32(32.0)
    corpus = build(squad, noise, sigma, layout)
    q = squad[qc] + np.float32(sigma) * qnoise
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    lib = _lib.load_library()
    dbg = lib.rr_debug_verify
    dbg.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    print(json.dumps({"state": ix.screen_state()}), flush=True)
    buf = (ctypes.c_ulonglong * 256)()
    prev = 0
    shown = 0
    for step in range(60):
        ix.search(q, 5)
        dbg(buf)
        b, fl, rr, ws = ix.screen_counts_all()
        if fl > prev:
            prev = fl
            for s in range(32):
                d = list(buf[s * 8:(s + 1) * 8])
                if d[5] == 2 or (d[5] == 1 and not d[6]):
                    print(json.dumps({"step": step, "slot": s, "kth_bound": f(d[0]), "tail_bound": f(d[1]),
                                      "ek1": f(d[2]), "ek2": f(d[3]), "nr": d[4], "decision": d[5],
                                      "complete": d[6]}), flush=True)
                    shown += 1
        if shown > 30:
            break
    print(json.dumps({"final": ix.screen_counts_all(), "state": ix.screen_state()}), flush=True)


if __name__ == "__main__":
    main()
