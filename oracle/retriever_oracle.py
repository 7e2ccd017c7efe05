"""ORACLE — CPU restatement (NumPy) of the reference retrieval hot path. TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only
as the checker / the timed CPU baseline. The product path (rag_service_amd, librag_retrieval.so) never
calls it; there is no CPU fallback.

Restated from ngray0/RAG-Serving-System @ 2025-07-04, rag_service/core/retriever.py:
  simple_retrieve        <- SimpleRetriever.retrieve        :78-128
  simple_batch_retrieve  <- SimpleRetriever.batch_retrieve  :131-166
  cosine_matrix          <- CupyRetriever.distance_cosine   :594-611  (NumPy in place of CuPy)
  cupy_retrieve          <- CupyRetriever.retrieve          :615-683
  cupy_batch_retrieve    <- CupyRetriever.batch_retrieve    :686-799
The restatement returns document INDICES (the reference returns documents[i]; tests run it with
documents = list(range(N)), so the two are the same thing).

Pinning: checked against golden vectors produced by the reference itself (imported in the build
container with a NumPy stand-in for its unused-at-runtime `cupy` import), tests/golden/make_golden.py ->
tests/golden/*.npz; see tests/test_oracle.py.

Arithmetic: the reference's scores come from OpenBLAS sgemv (SimpleRetriever, numpy 2.2.x) and cuBLAS
SGEMM (CupyRetriever). The restatement uses the same NumPy calls, so on this image it reproduces
SimpleRetriever bit-for-bit. Ties between equal scores are ordered as numpy's argpartition/argsort
happen to order them (implementation defined); `canonical_topk` gives the deterministic
(score desc, index asc) order the HIP path implements.
"""
from __future__ import annotations

import numbers
from typing import List, Optional, Sequence, Tuple

import numpy as np


# --------------------------------------------------------------------------------------------------
# SimpleRetriever (dot product)
# --------------------------------------------------------------------------------------------------
def simple_retrieve(doc: np.ndarray, query_emb: np.ndarray, k: int = 2) -> List[int]:
    """retriever.py:78-128 — returns top-k indices (descending score) or [] on the reference's errors."""
    if doc.dtype != np.float32:                       # :71-73 (constructor cast)
        doc = doc.astype(np.float32)
    if k <= 0:                                        # :89-91
        return []
    if k > doc.shape[0]:                              # :92-94
        k = doc.shape[0]
    try:
        if query_emb.dtype != np.float32:             # :98-99
            query_emb = query_emb.astype(np.float32)
        if query_emb.ndim != 1:                       # :100-106
            if query_emb.ndim == 2 and query_emb.shape[0] == 1:
                query_emb = query_emb.flatten()
            else:
                return []
        if query_emb.shape[0] != doc.shape[1]:        # :108-110
            return []
        sims = doc @ query_emb                        # :112
        top = np.argpartition(sims, -k)[-k:]          # :118
        top = top[np.argsort(sims[top])[::-1]]        # :120
        return [int(i) for i in top]
    except Exception:                                 # :126-128
        return []


def simple_batch_retrieve(doc: np.ndarray, queries: np.ndarray, ks: Sequence[int]) -> List[List[int]]:
    """retriever.py:131-166 — per-query loop over simple_retrieve."""
    if queries.ndim != 2:                             # :146-149
        return [[] for _ in ks]
    if queries.shape[0] != len(ks):                   # :150-153
        return [[] for _ in ks]
    if queries.shape[1] != doc.shape[1]:              # :154-156
        return [[] for _ in ks]
    return [simple_retrieve(doc, q, ks[i]) for i, q in enumerate(queries)]   # :159-164


# --------------------------------------------------------------------------------------------------
# CupyRetriever (clipped cosine), CuPy replaced by NumPy
# --------------------------------------------------------------------------------------------------
def cosine_matrix(X: np.ndarray, Y: np.ndarray, epsilon: float = 1e-8,
                  y_norms: Optional[np.ndarray] = None) -> np.ndarray:
    """retriever.py:594-611: dot / (|x| |y|^T + eps), clipped to [-1, 1], fp32 throughout."""
    X = np.asarray(X, dtype=np.float32)
    Y = np.asarray(Y, dtype=np.float32)
    dot = X @ Y.T                                                  # :600
    nx = np.linalg.norm(X, axis=1, keepdims=True)                  # :602
    ny = np.linalg.norm(Y, axis=1, keepdims=True) if y_norms is None else y_norms.reshape(-1, 1)  # :603
    nprod = nx @ ny.T                                              # :605
    cos = dot / (nprod + np.float32(epsilon))                     # :607
    return np.clip(cos, -1.0, 1.0)                                 # :609


def cupy_retrieve(doc: np.ndarray, query_emb, k: int = 2) -> List[int]:
    """retriever.py:615-683."""
    if not isinstance(query_emb, np.ndarray):                     # :629-631
        return []
    if query_emb.ndim == 2 and query_emb.shape[0] == 1:            # :632-634
        query_emb = query_emb.flatten()
    elif query_emb.ndim != 1:                                      # :635-637
        return []
    if query_emb.shape[0] != doc.shape[1]:                         # :638-640
        return []
    n = doc.shape[0]
    actual_k = min(k, n)                                           # :643
    if actual_k <= 0:                                              # :644-646
        return []
    try:
        q = query_emb.astype(np.float32).reshape(1, -1)            # :650-652
        scores = cosine_matrix(q, doc)[0]                          # :656-657
        part = np.argpartition(scores, n - actual_k)[-actual_k:]   # :662
        order = np.argsort(-scores[part])                          # :668
        return [int(i) for i in part[order]]                       # :669-675
    except Exception:                                              # :681-683
        return []


def cupy_batch_retrieve(doc: np.ndarray, queries, ks) -> List[List[int]]:
    """retriever.py:686-799 (including the strict isinstance(k, int) rule, :720-722)."""
    batch_size = queries.shape[0]                                  # :702 (before the type check)
    if not isinstance(queries, np.ndarray):                        # :705-707
        return [[] for _ in ks]
    if queries.ndim != 2:                                          # :708-710
        return [[] for _ in ks]
    if batch_size == 0:                                            # :711-713
        return []
    if not isinstance(ks, list) or batch_size != len(ks):          # :714-716
        return [[] for _ in range(batch_size)]
    if queries.shape[1] != doc.shape[1]:                           # :717-719
        return [[] for _ in ks]
    if not all(isinstance(k_val, int) for k_val in ks):            # :720-722
        return [[] for _ in ks]
    n = doc.shape[0]
    valid_ks = [k_val for k_val in ks if k_val > 0]                # :725-728
    if not valid_ks:
        return [[] for _ in ks]
    max_k = min(max(valid_ks), n)                                  # :729-730
    if max_k <= 0:
        return [[] for _ in ks]
    try:
        q = queries.astype(np.float32)                             # :736-738
        scores = cosine_matrix(q, doc)                             # :742
        top = np.empty((batch_size, max_k), dtype=np.int64)        # :746
        for i in range(batch_size):                                # :750-769
            row = scores[i]
            part = np.argpartition(row, n - max_k)[-max_k:]
            order = np.argsort(-row[part])
            final = part[order]
            top[i, :final.shape[0]] = final
            if final.shape[0] < max_k:
                top[i, final.shape[0]:] = -1
        out = []
        for i in range(batch_size):                                # :777-790
            k_i = ks[i]
            if k_i <= 0:
                out.append([])
                continue
            row = top[i]
            out.append([int(j) for j in row[row >= 0][:k_i]])
        return out
    except Exception:                                              # :796-799
        return [[] for _ in ks]


# --------------------------------------------------------------------------------------------------
# scoring helpers for parity checks (not reference code paths)
# --------------------------------------------------------------------------------------------------
def exact_scores(doc: np.ndarray, queries: np.ndarray, metric: str) -> np.ndarray:
    """fp64 evaluation of the metric: dot, or dot/(|q||d| + 1e-8) clipped (the reference's formula)."""
    d64 = doc.astype(np.float64)
    q64 = np.atleast_2d(queries).astype(np.float64)
    dot = q64 @ d64.T
    if metric == "dot":
        return dot
    nq = np.linalg.norm(q64, axis=1, keepdims=True)
    nd = np.linalg.norm(d64, axis=1, keepdims=True)
    return np.clip(dot / (nq @ nd.T + 1e-8), -1.0, 1.0)


def canonical_topk(scores: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Top-k of each row by (score desc, index asc) — the HIP path's deterministic tie rule.
    Rows shorter than k are padded with (-inf, -1)."""
    scores = np.atleast_2d(scores)
    b, n = scores.shape
    kk = min(k, n)
    idx = np.empty((b, k), dtype=np.int64)
    val = np.empty((b, k), dtype=scores.dtype)
    for i in range(b):
        order = np.lexsort((np.arange(n), -scores[i]))[:kk]
        idx[i, :kk] = order
        val[i, :kk] = scores[i, order]
    idx[:, kk:] = -1
    val[:, kk:] = -np.inf
    return val, idx


def topk_gap(scores: np.ndarray, k: int) -> float:
    """Smallest gap between consecutive sorted scores among the top k+1 of any row (ties -> 0)."""
    scores = np.atleast_2d(scores)
    k1 = min(k + 1, scores.shape[1])
    part = -np.sort(-scores, axis=1)[:, :k1]
    if k1 < 2:
        return float("inf")
    return float(np.min(part[:, :-1] - part[:, 1:]))


def is_integral(k) -> bool:
    return isinstance(k, (numbers.Integral, np.integer))
