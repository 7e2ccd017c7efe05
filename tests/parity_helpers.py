"""Comparison helpers shared by the parity tests (test infrastructure)."""
from __future__ import annotations

import numpy as np

from oracle.retriever_oracle import exact_scores

SCORE_TOL = 1e-3      # north-star tolerance on returned scores (fp32)
NEAR_TIE = 2e-6       # fp64 score gap below which two fp32 pipelines may legitimately order docs differently


def check_topk(got_idx, got_scores, ref_idx, corpus, queries, metric, near_tie=NEAR_TIE, score_tol=SCORE_TOL):
    """Assert the HIP top-k equals the reference's.

    * every returned score is within `score_tol` of the fp64 value of the metric at that index;
    * per query, the index list equals the reference's exactly, except where the two lists differ only
      between documents whose fp64 scores are within `near_tie` (numerically tied; reported).
    Returns (exact_rows, near_tie_rows).
    """
    got_idx = np.asarray(got_idx)
    ref_idx = np.asarray(ref_idx)
    assert got_idx.shape == ref_idx.shape, (got_idx.shape, ref_idx.shape)
    valid = got_idx >= 0
    assert np.array_equal(valid, ref_idx >= 0)
    exact = exact_scores(corpus, queries, metric)
    if got_scores is not None:
        at = np.take_along_axis(exact, np.maximum(got_idx, 0), axis=1)
        err = np.abs(np.where(valid, at - np.asarray(got_scores, dtype=np.float64), 0.0))
        assert err.max() <= score_tol, f"score error {err.max()}"
    exact_rows = near_rows = 0
    for i in range(got_idx.shape[0]):
        if np.array_equal(got_idx[i], ref_idx[i]):
            exact_rows += 1
            continue
        g = exact[i, got_idx[i][valid[i]]]
        r = exact[i, ref_idx[i][valid[i]]]
        assert np.all(np.abs(g - r) <= near_tie), (
            f"query {i}: got {got_idx[i].tolist()} ref {ref_idx[i].tolist()} scores {g} vs {r}")
        near_rows += 1
    return exact_rows, near_rows
