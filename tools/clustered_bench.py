#!/usr/bin/env python3
"""The screened search on realistic, clustered embeddings.

The only real embeddings the reference ships are data/squad_embeddings.npy (1000 e5-large rows; committed as
tests/golden/data/squad_embeddings.npy). A 1M-row corpus is built from them: row i = the SQuAD row c(i) plus seeded
Gaussian noise of relative size sigma, L2-normalised; queries = other noisy copies of SQuAD rows (B = 32). Two
layouts: "interleaved" (c(i) = i mod 1000: each cluster spread over the whole corpus) and "contiguous"
(c(i) = i div 1000: each cluster one run of 1000 rows, i.e. inside a few workgroups' chunks).

For each (sigma, layout), k = 5 cosine (the headline's search), on one GPU:
  * screened (RR_KERNEL_AUTO, after W awaited warm-up steps in which the adaptive screen settles: short -> full
    per-lane lists, or a pause to the exact kernel): q/s over K staged steps with every flagged block's exact re-run
    paid inside the timed window (bench.timed_steps), the flagged-block rate, the slots the verify's wide phase
    proved, the screen's adaptive state;
  * exact (RR_KERNEL_EXACT, one pass over the fp32 rows): q/s;
  * results of a fetched search: screened == exact, bit for bit.
One JSON line per configuration, then a summary line.

    python tools/clustered_bench.py [--docs 1000000] [--steps 100] [--sigmas 0.01,0.03,0.1,0.3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "rag-serving-system_amd"))


def build(squad: np.ndarray, noise: np.ndarray, sigma: float, layout: str) -> np.ndarray:
    n, d = noise.shape
    c = np.arange(n) % squad.shape[0] if layout == "interleaved" else np.arange(n) // (n // squad.shape[0])
    c = np.minimum(c, squad.shape[0] - 1)
    out = squad[c]
    out += np.float32(sigma) * noise
    out /= np.linalg.norm(out, axis=1, keepdims=True)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=80,
                    help="untimed steps first, each awaited: the adaptive screen settles (short -> full lists, pause)")
    ap.add_argument("--sigmas", default="0.01,0.03,0.1,0.3")
    ap.add_argument("--layouts", default="interleaved,contiguous")
    ap.add_argument("--int8", default="auto", choices=["auto", "off"],
                    help="off: screen the f16 copy (rr_screen_int8(0)) instead of the int8 one")
    args = ap.parse_args()

    import bench
    from rag_service_amd import Index

    squad = np.load(os.path.join(REPO, "tests", "golden", "data", "squad_embeddings.npy")).astype(np.float32)
    squad /= np.linalg.norm(squad, axis=1, keepdims=True)
    d = squad.shape[1]
    rng = np.random.default_rng(20260)
    t = time.perf_counter()
    noise = rng.standard_normal((args.docs, d), dtype=np.float32) / np.float32(np.sqrt(d))   # |noise| ~ 1
    qrng = np.random.default_rng(777)
    qc = qrng.integers(0, squad.shape[0], args.batch)
    qnoise = qrng.standard_normal((args.batch, d), dtype=np.float32) / np.float32(np.sqrt(d))
    print(json.dumps({"setup_s": round(time.perf_counter() - t, 1)}), flush=True)

    def cuda_sync():
        return None

    ix = Index(dtype="fp32", metric="cosine")
    rows = []
    for layout in args.layouts.split(","):
        for sigma in [float(x) for x in args.sigmas.split(",")]:
            corpus = build(squad, noise, sigma, layout)
            q = squad[qc] + np.float32(sigma) * qnoise
            q /= np.linalg.norm(q, axis=1, keepdims=True)
            ix.set_kernel("auto")
            ix.load(corpus)
            if args.int8 == "off":
                ix.screen_int8(False)
            del corpus
            ix.set_queries(q)
            # warm-up paced like a serving loop (each batch's results awaited): the adaptive screen decides from the
            # counts of COMPLETED blocks, which an unpaced burst of staged searches outruns
            for _ in range(args.warmup):
                ix.search_staged(args.k)
                ix.synchronize()
            acct = {}
            s_el, _, _ = bench.timed_steps(ix, args.k, args.steps, 0, None, cuda_sync, 10, acct)
            state = ix.screen_state()
            i8 = ix.screen_int8()   # (the int8 copy gives way to the f16 one when it re-runs blocks)
            got = ix.search(q, args.k)
            ix.set_kernel("exact")
            ix.set_queries(q)
            e_el, _, _ = bench.timed_steps(ix, args.k, args.steps, args.warmup, None, cuda_sync, 10)
            want = ix.search(q, args.k)
            ix.set_kernel("auto")
            same = bool(np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]))
            # how crowded the top is: exact scores of the k-th and of the 16th / 32nd candidates (the list widths)
            ix.set_kernel("exact")
            s32, _ = ix.search(q, 32)
            ix.set_kernel("auto")
            gap16 = float(np.median(s32[:, args.k - 1] - s32[:, 15]))
            gap32 = float(np.median(s32[:, args.k - 1] - s32[:, 31]))
            rec = {"layout": layout, "sigma": sigma, "docs": args.docs, "k": args.k, "batch": args.batch,
                   "screened_qps": round(args.batch * args.steps / s_el, 1),
                   "exact_qps": round(args.batch * args.steps / e_el, 1),
                   "speedup": round(e_el / s_el, 3),
                   "flagged_blocks": acct["flagged"], "blocks": acct["blocks"],
                   "reruns_paid": acct["reruns_paid"], "reruns_library": acct["reruns_library"],
                   "flag_rate": round(acct["flagged"] / max(1, acct["blocks"]), 4),
                   "wide_verified_slots": acct["wide_slots"],
                   "screen_state_after": dict(zip(("repair_mode", "pause_left", "pauses"), state), int8=i8),
                   "repaired_slots": ix.screen_repairs(),
                   "bit_identical_to_exact": same,
                   "median_score_gap_k_to_16": round(gap16, 6), "median_score_gap_k_to_32": round(gap32, 6),
                   "top1_median": round(float(np.median(s32[:, 0])), 5)}
            rows.append(rec)
            print(json.dumps(rec), flush=True)
    ix.close()
    print(json.dumps({"summary": [(r["layout"], r["sigma"], r["flag_rate"], r["speedup"]) for r in rows],
                      "all_bit_identical": all(r["bit_identical_to_exact"] for r in rows)}), flush=True)


if __name__ == "__main__":
    main()
