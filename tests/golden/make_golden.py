"""Generate golden vectors by running the REFERENCE retrievers themselves (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--big]

The reference module (rag_service/core/retriever.py) imports `cupy` at top level (:9), which is not
installed here. We register a small NumPy-backed stand-in under that name before importing it, so:
  * SimpleRetriever runs its own code verbatim (it never touches cupy): the primary oracle pin;
  * CupyRetriever runs its own control flow with NumPy arithmetic in place of CuPy/cuBLAS.
Documents are list(range(N)), so the "documents" the reference returns are row indices.

Only data comes out of this script (tests/golden/*.npz, *.json): inputs are described by seeds or by
the reference's own data files (copied under tests/golden/data/), outputs are the reference's index
lists plus fp64 scores recomputed at those indices. /root/reference is never needed at test time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from oracle import synth  # noqa: E402
from oracle.retriever_oracle import exact_scores, topk_gap  # noqa: E402


def install_cupy_standin() -> None:
    class _DevArray(np.ndarray):
        def get(self):
            return np.asarray(self)

    def _wrap(x):
        return np.asarray(x).view(_DevArray) if isinstance(x, np.ndarray) else x

    cp = types.ModuleType("cupy")
    cp.ndarray = _DevArray
    cp.asarray = lambda x, dtype=None: np.asarray(x, dtype=dtype).view(_DevArray)
    cp.empty = lambda shape, dtype=float: np.empty(shape, dtype=dtype).view(_DevArray)
    cp.argpartition = lambda a, kth, axis=-1: _wrap(np.argpartition(a, kth, axis=axis))
    cp.argsort = lambda a, axis=-1: _wrap(np.argsort(a, axis=axis))
    cp.clip = lambda a, lo, hi: _wrap(np.clip(a, lo, hi))
    cp.int64, cp.float32, cp.float64 = np.int64, np.float32, np.float64
    linalg = types.ModuleType("cupy.linalg")
    linalg.norm = lambda x, ord=None, axis=None, keepdims=False: _wrap(
        np.linalg.norm(x, ord=ord, axis=axis, keepdims=keepdims))
    cp.linalg = linalg
    sys.modules["cupy"] = cp
    sys.modules["cupy.linalg"] = linalg


def import_reference():
    install_cupy_standin()
    sys.path.insert(0, REF)
    import importlib
    mod = importlib.import_module("rag_service.core.retriever")
    import logging
    logging.getLogger().setLevel(logging.ERROR)
    return mod


def pad_lists(lists, width):
    out = np.full((len(lists), width), -1, dtype=np.int64)
    for i, l in enumerate(lists):
        out[i, :len(l)] = l
    return out


def run_case(ref, corpus, queries, k, name, out, metric_both=True, dtype_note="fp32"):
    """Reference SimpleRetriever + CupyRetriever on (corpus, queries, k) -> arrays in `out`."""
    n = corpus.shape[0]
    docs = list(range(n))
    t0 = time.time()
    simple = ref.SimpleRetriever(doc_embeddings=corpus, documents=docs)
    s_lists = simple.batch_retrieve(queries, [k] * queries.shape[0])
    t1 = time.time()
    kk = min(k, n)
    out[f"{name}_simple_idx"] = pad_lists(s_lists, kk)
    sd = exact_scores(corpus, queries, "dot")
    out[f"{name}_simple_gap"] = np.float64(topk_gap(sd.astype(np.float32), kk))
    out[f"{name}_simple_score"] = np.take_along_axis(sd, np.maximum(out[f"{name}_simple_idx"], 0), axis=1)
    if metric_both:
        cupy = ref.CupyRetriever(doc_embeddings=corpus, documents=docs)
        c_lists = cupy.batch_retrieve(queries, [k] * queries.shape[0])
        out[f"{name}_cupy_idx"] = pad_lists(c_lists, kk)
        sc = exact_scores(corpus, queries, "cosine")
        out[f"{name}_cupy_gap"] = np.float64(topk_gap(sc.astype(np.float32), kk))
        out[f"{name}_cupy_score"] = np.take_along_axis(sc, np.maximum(out[f"{name}_cupy_idx"], 0), axis=1)
    print(f"  {name}: n={n} b={queries.shape[0]} k={k} simple {t1 - t0:.2f}s total {time.time() - t0:.2f}s "
          f"gap={float(out[f'{name}_simple_gap']):.3g}", flush=True)


def edge_cases(ref, corpus):
    """Outputs of the reference's validation / clamping paths."""
    n, d = corpus.shape
    docs = list(range(n))
    simple = ref.SimpleRetriever(doc_embeddings=corpus, documents=docs)
    cupy = ref.CupyRetriever(doc_embeddings=corpus, documents=docs)
    rng = np.random.default_rng(7)
    q4 = rng.standard_normal((4, d)).astype(np.float32)
    q4 /= np.linalg.norm(q4, axis=1, keepdims=True)
    cases = {}
    cases["mixed_ks"] = {"ks": [3, 0, -1, 7], "simple": simple.batch_retrieve(q4, [3, 0, -1, 7]),
                         "cupy": cupy.batch_retrieve(q4, [3, 0, -1, 7])}
    cases["k_gt_n"] = {"ks": [n + 50, 2, n, 1], "simple": simple.batch_retrieve(q4, [n + 50, 2, n, 1]),
                       "cupy": cupy.batch_retrieve(q4, [n + 50, 2, n, 1])}
    cases["all_nonpositive"] = {"ks": [0, -3, 0, -1], "simple": simple.batch_retrieve(q4, [0, -3, 0, -1]),
                                "cupy": cupy.batch_retrieve(q4, [0, -3, 0, -1])}
    cases["float64_queries"] = {"ks": [5, 5, 5, 5], "simple": simple.batch_retrieve(q4.astype(np.float64), [5] * 4),
                                "cupy": cupy.batch_retrieve(q4.astype(np.float64), [5] * 4)}
    cases["wrong_dim"] = {"ks": [5, 5, 5, 5], "simple": simple.batch_retrieve(q4[:, :d - 8], [5] * 4),
                          "cupy": cupy.batch_retrieve(q4[:, :d - 8], [5] * 4)}
    cases["np_int64_ks"] = {"ks": [5, 5, 5, 5], "simple": simple.batch_retrieve(q4, [np.int64(5)] * 4),
                            "cupy": cupy.batch_retrieve(q4, [np.int64(5)] * 4)}
    cases["len_mismatch"] = {"ks": [5, 5, 5], "simple": simple.batch_retrieve(q4, [5, 5, 5]),
                             "cupy": cupy.batch_retrieve(q4, [5, 5, 5])}
    cases["empty_batch"] = {"ks": [], "simple": simple.batch_retrieve(q4[:0], []),
                            "cupy": cupy.batch_retrieve(q4[:0], [])}
    cases["one_d_batch"] = {"ks": [5], "simple": simple.batch_retrieve(q4[0], [5]),
                            "cupy": cupy.batch_retrieve(q4[0], [5])}
    # single-query entry points
    cases["retrieve_1d"] = {"k": 3, "simple": simple.retrieve(q4[0], 3), "cupy": cupy.retrieve(q4[0], 3)}
    cases["retrieve_1xd"] = {"k": 3, "simple": simple.retrieve(q4[:1], 3), "cupy": cupy.retrieve(q4[:1], 3)}
    cases["retrieve_k0"] = {"k": 0, "simple": simple.retrieve(q4[0], 0), "cupy": cupy.retrieve(q4[0], 0)}
    cases["retrieve_kneg"] = {"k": -2, "simple": simple.retrieve(q4[0], -2), "cupy": cupy.retrieve(q4[0], -2)}
    cases["retrieve_k_gt_n"] = {"k": n + 3, "simple": simple.retrieve(q4[0], n + 3), "cupy": cupy.retrieve(q4[0], n + 3)}
    cases["retrieve_2xd"] = {"k": 3, "simple": simple.retrieve(q4[:2], 3), "cupy": cupy.retrieve(q4[:2], 3)}
    cases["retrieve_wrong_dim"] = {"k": 3, "simple": simple.retrieve(q4[0, :d - 8], 3),
                                   "cupy": cupy.retrieve(q4[0, :d - 8], 3)}
    cases["retrieve_np_int64_k"] = {"k": 3, "simple": simple.retrieve(q4[0], np.int64(3)),
                                    "cupy": cupy.retrieve(q4[0], np.int64(3))}
    cases["retrieve_float_k"] = {"k": 2.5, "simple": simple.retrieve(q4[0], 2.5), "cupy": cupy.retrieve(q4[0], 2.5)}
    cases["retrieve_float64"] = {"k": 4, "simple": simple.retrieve(q4[0].astype(np.float64), 4),
                                 "cupy": cupy.retrieve(q4[0].astype(np.float64), 4)}
    try:
        cupy.batch_retrieve(q4.tolist(), [5] * 4)
        cases["cupy_list_input"] = "no-exception"
    except Exception as e:  # the reference reads .shape before its type check (:702)
        cases["cupy_list_input"] = type(e).__name__
    return {"seed": 7, "n": n, "d": d, "cases": cases}


def streaming_topk(chunks, queries, metric, k):
    """fp64 canonical top-(k+1) over row chunks [(row0, rows)], without the full B x N score matrix."""
    b = queries.shape[0]
    best_s = np.full((b, 0), -np.inf)
    best_i = np.full((b, 0), -1, dtype=np.int64)
    for r0, x in chunks:
        s = exact_scores(x, queries, metric)
        cs = np.concatenate([best_s, s], axis=1)
        ci = np.concatenate([best_i, np.broadcast_to(np.arange(r0, r0 + x.shape[0]), s.shape)], axis=1)
        keep = np.empty((b, min(k + 1, cs.shape[1])), dtype=np.int64)
        for i in range(b):
            keep[i] = np.lexsort((ci[i], -cs[i]))[:keep.shape[1]]
        best_s = np.take_along_axis(cs, keep, axis=1)
        best_i = np.take_along_axis(ci, keep, axis=1)
    return best_s, best_i


def config_goldens(ref):
    """BASELINE.json configs 3 and 5 at (or toward) their defining shapes, from the reference's own retrievers.

    config 3: F2 exact-integer 10M x 1024 (seed 1234), 32 queries (seed 99), k=10. SimpleRetriever (dot) runs on
      the whole corpus. CupyRetriever (cosine) would materialise a 10M x 1024 temporary in its corpus norm, more
      than this container holds, so it runs on 1M-row chunks (its own code on each), and the chunk winners are
      merged by fp64 cosine: the global top-10 lies in the union of chunk top-10s; the merge order can differ
      from the reference's fp32 order only inside the recorded gap.
    config 5: bf16-rounded F3 unit-norm 1M x 1024 (seed 1234), 64 queries (seed 4321), k=10, both retrievers on
      the whole corpus (config 5 defines 50M rows over 8 GPUs; 1M is the largest the host-side reference pin
      reaches in minutes here; the device tests use 8 shards of it)."""
    out = {}
    n3, d, k = 10_000_000, 1024, 10
    t0 = time.time()
    corpus = np.empty((n3, d), dtype=np.float32)
    step = 1 << 20
    for r0 in range(0, n3, step):
        corpus[r0:r0 + step] = synth.exact_int_rows(1234, r0, min(step, n3 - r0), d)
        print(f"  F2 rows {r0 + step} ({time.time() - t0:.0f}s)", flush=True)
    q = synth.exact_int_queries(99, 32, d)
    docs = list(range(n3))
    simple = ref.SimpleRetriever(doc_embeddings=corpus, documents=docs)
    out["c3_simple_idx"] = pad_lists(simple.batch_retrieve(q, [k] * 32), k)
    chunks = [(r0, corpus[r0:r0 + step]) for r0 in range(0, n3, step)]
    s, i = streaming_topk(chunks, q, "dot", k)
    out["c3_simple_score"] = np.stack([exact_scores(corpus[out["c3_simple_idx"][qi]], q[qi:qi + 1], "dot")[0]
                                       for qi in range(32)])
    out["c3_simple_gap"] = np.float64(np.min(s[:, :-1] - s[:, 1:]))
    cand = [[] for _ in range(32)]
    for r0, x in chunks:
        cupy = ref.CupyRetriever(doc_embeddings=x, documents=list(range(r0, r0 + x.shape[0])))
        for qi, lst in enumerate(cupy.batch_retrieve(q, [k] * 32)):
            cand[qi].extend(lst)
    s, i = streaming_topk(chunks, q, "cosine", k)
    out["c3_cupy_gap"] = np.float64(np.min(s[:, :-1] - s[:, 1:]))
    idx = np.full((32, k), -1, dtype=np.int64)
    for qi in range(32):
        c = np.array(sorted(set(cand[qi])), dtype=np.int64)
        cs = exact_scores(corpus[c], q[qi:qi + 1], "cosine")[0]
        idx[qi] = c[np.lexsort((c, -cs))[:k]]
    out["c3_cupy_idx"] = idx
    out["c3_cupy_score"] = np.stack([exact_scores(corpus[idx[qi]], q[qi:qi + 1], "cosine")[0] for qi in range(32)])
    out["c3_meta"] = np.array([1234, 99, n3, d, k], dtype=np.int64)
    print(f"  config 3 done ({time.time() - t0:.0f}s) gaps dot {float(out['c3_simple_gap']):.3g} "
          f"cos {float(out['c3_cupy_gap']):.3g}", flush=True)
    del simple, chunks, corpus, docs, cupy, x    # (a chunk view would keep the 41 GB corpus alive)
    np.savez_compressed(os.path.join(HERE, "golden_configs.npz"), **out)

    n5 = 1_000_000
    c5 = synth.bf16_round(synth.unit_norm_gaussian(1234, n5, d))
    q5 = synth.unit_norm_gaussian(4321, 64, d)
    run_case(ref, c5, q5, k, "c5", out)
    out["c5_meta"] = np.array([1234, 4321, n5, d, k], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "golden_configs.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true", help="also the 1M-row cases (needs ~20 GB RAM, minutes)")
    ap.add_argument("--configs", action="store_true",
                    help="only the BASELINE config 3/5 goldens (golden_configs.npz; ~50 GB RAM, ~15 min)")
    args = ap.parse_args()
    ref = import_reference()
    print("reference imported:", ref.__file__, flush=True)
    if args.configs:
        config_goldens(ref)
        print("done", flush=True)
        return

    # ---- F1: the reference's own data files --------------------------------------------------
    sf = np.load(os.path.join(HERE, "data", "short_facts_embeddings.npy"))
    sq = np.load(os.path.join(HERE, "data", "squad_embeddings.npy"))
    out = {}
    rng = np.random.default_rng(0)
    qr = rng.standard_normal((32, 1024)).astype(np.float32)
    qr /= np.linalg.norm(qr, axis=1, keepdims=True)
    for k in (1, 5, 10):
        run_case(ref, sf, sf, k, f"sf_self_k{k}", out)
        run_case(ref, sf, qr, k, f"sf_rand_k{k}", out)
    run_case(ref, sf, qr, 100, "sf_rand_k100", out)
    for k in (2, 5, 10, 32):
        run_case(ref, sq, qr, k, f"sq_rand_k{k}", out)
    run_case(ref, sq, sq[:64], 5, "sq_self_k5", out)
    run_case(ref, sq, qr, 40, "sq_rand_k40", out)
    # mixed-sign unnormalised queries (raw dot differs from cosine ranking)
    qm = (rng.standard_normal((32, 1024)) * rng.uniform(0.1, 3.0, size=(32, 1))).astype(np.float32)
    run_case(ref, sq, qm, 10, "sq_scaled_k10", out)
    out["rand_queries"] = qr
    out["scaled_queries"] = qm
    np.savez_compressed(os.path.join(HERE, "golden_data.npz"), **out)
    with open(os.path.join(HERE, "golden_edge_cases.json"), "w") as f:
        json.dump(edge_cases(ref, sf), f, indent=1)

    # ---- F2 / F3 synthetic ------------------------------------------------------------------------
    syn = {}
    n_small = 65536
    c2 = synth.exact_int_rows(1234, 0, n_small, 1024)
    q2 = synth.exact_int_queries(99, 32, 1024)
    run_case(ref, c2, q2, 10, "f2_64k_k10", syn)
    c3 = synth.unit_norm_gaussian(1234, n_small, 1024)
    q3 = synth.unit_norm_gaussian(5678, 32, 1024)
    run_case(ref, c3, q3, 10, "f3_64k_k10", syn)
    run_case(ref, synth.bf16_round(c3), q3, 10, "f3bf_64k_k10", syn)
    syn["meta"] = np.array([1234, 99, 5678, n_small], dtype=np.int64)
    if args.big:
        n_big = 1_000_000
        del c2, c3
        c2 = synth.exact_int_rows(1234, 0, n_big, 1024)
        run_case(ref, c2, q2, 5, "f2_1m_k5", syn, metric_both=False)
        run_case(ref, c2, q2, 10, "f2_1m_k10", syn, metric_both=False)
        del c2
        c3 = synth.unit_norm_gaussian(1234, n_big, 1024)
        run_case(ref, c3, q3, 5, "f3_1m_k5", syn)
        run_case(ref, c3, q3, 10, "f3_1m_k10", syn)
        c3 = synth.bf16_round(c3)
        run_case(ref, c3, q3, 10, "f3bf_1m_k10", syn, metric_both=False)
    np.savez_compressed(os.path.join(HERE, "golden_synth.npz"), **syn)
    print("done", flush=True)


if __name__ == "__main__":
    main()
