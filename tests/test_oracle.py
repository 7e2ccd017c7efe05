"""The oracle (CPU restatement) pinned against the reference's own outputs (golden vectors)."""
import numpy as np
import pytest

from oracle import synth
from oracle.retriever_oracle import (canonical_topk, cupy_batch_retrieve, cupy_retrieve, exact_scores,
                                     simple_batch_retrieve, simple_retrieve)

CASES = [
    ("sf_self_k1", "sf", "sf_self", 1), ("sf_self_k5", "sf", "sf_self", 5), ("sf_self_k10", "sf", "sf_self", 10),
    ("sf_rand_k1", "sf", "rand", 1), ("sf_rand_k5", "sf", "rand", 5), ("sf_rand_k10", "sf", "rand", 10),
    ("sf_rand_k100", "sf", "rand", 100), ("sq_rand_k2", "sq", "rand", 2), ("sq_rand_k5", "sq", "rand", 5),
    ("sq_rand_k10", "sq", "rand", 10), ("sq_rand_k32", "sq", "rand", 32), ("sq_rand_k40", "sq", "rand", 40),
    ("sq_self_k5", "sq", "sq_self", 5), ("sq_scaled_k10", "sq", "scaled", 10),
]


def _inputs(ck, qk, short_facts, squad, g):
    corpus = short_facts if ck == "sf" else squad
    q = {"sf_self": short_facts, "sq_self": squad[:64], "rand": g["rand_queries"], "scaled": g["scaled_queries"]}[qk]
    return corpus, q


@pytest.mark.parametrize("name,ck,qk,k", CASES)
def test_oracle_reproduces_reference(golden_data, short_facts, squad, name, ck, qk, k):
    corpus, q = _inputs(ck, qk, short_facts, squad, golden_data)
    s = simple_batch_retrieve(corpus, q, [k] * q.shape[0])
    c = cupy_batch_retrieve(corpus, q, [k] * q.shape[0])
    assert s == golden_data[f"{name}_simple_idx"].tolist()
    assert c == golden_data[f"{name}_cupy_idx"].tolist()


def test_oracle_synthetic_64k(golden_synth):
    seed, qseed2, qseed3, n = [int(x) for x in golden_synth["meta"]]
    c2 = synth.exact_int_rows(seed, 0, n, 1024)
    q2 = synth.exact_int_queries(qseed2, 32, 1024)
    assert simple_batch_retrieve(c2, q2, [10] * 32) == golden_synth["f2_64k_k10_simple_idx"].tolist()
    c3 = synth.unit_norm_gaussian(seed, n, 1024)
    q3 = synth.unit_norm_gaussian(qseed3, 32, 1024)
    assert simple_batch_retrieve(c3, q3, [10] * 32) == golden_synth["f3_64k_k10_simple_idx"].tolist()
    assert cupy_batch_retrieve(c3, q3, [10] * 32) == golden_synth["f3_64k_k10_cupy_idx"].tolist()
    c3b = synth.bf16_round(c3)
    assert simple_batch_retrieve(c3b, q3, [10] * 32) == golden_synth["f3bf_64k_k10_simple_idx"].tolist()


def test_oracle_edge_cases(golden_edges, short_facts):
    n, d = short_facts.shape
    rng = np.random.default_rng(golden_edges["seed"])
    q4 = rng.standard_normal((4, d)).astype(np.float32)
    q4 /= np.linalg.norm(q4, axis=1, keepdims=True)
    c = golden_edges["cases"]
    batch = {"mixed_ks": (q4, [3, 0, -1, 7]), "k_gt_n": (q4, [n + 50, 2, n, 1]),
             "all_nonpositive": (q4, [0, -3, 0, -1]), "float64_queries": (q4.astype(np.float64), [5] * 4),
             "wrong_dim": (q4[:, :d - 8], [5] * 4), "np_int64_ks": (q4, [np.int64(5)] * 4),
             "len_mismatch": (q4, [5, 5, 5]), "empty_batch": (q4[:0], []), "one_d_batch": (q4[0], [5])}
    for case, (q, ks) in batch.items():
        assert simple_batch_retrieve(short_facts, q, ks) == c[case]["simple"], case
        assert cupy_batch_retrieve(short_facts, q, ks) == c[case]["cupy"], case
    single = {"retrieve_1d": (q4[0], 3), "retrieve_1xd": (q4[:1], 3), "retrieve_k0": (q4[0], 0),
              "retrieve_kneg": (q4[0], -2), "retrieve_k_gt_n": (q4[0], n + 3), "retrieve_2xd": (q4[:2], 3),
              "retrieve_wrong_dim": (q4[0, :d - 8], 3), "retrieve_np_int64_k": (q4[0], np.int64(3)),
              "retrieve_float_k": (q4[0], 2.5), "retrieve_float64": (q4[0].astype(np.float64), 4)}
    for case, (q, k) in single.items():
        assert simple_retrieve(short_facts, q, k) == c[case]["simple"], case
        assert cupy_retrieve(short_facts, q, k) == c[case]["cupy"], case


def test_exact_integer_corpus_is_exact_in_fp32():
    c = synth.exact_int_rows(5, 0, 2000, 1024)
    q = synth.exact_int_queries(6, 4, 1024)
    assert np.array_equal((q @ c.T).astype(np.float64), q.astype(np.float64) @ c.astype(np.float64).T)
    assert np.array_equal(synth.bf16_round(c), c)


def test_generators_are_chunk_invariant():
    a = synth.exact_int_rows(9, 100, 300, 128, chunk_rows=7)
    b = synth.exact_int_rows(9, 0, 400, 128)[100:]
    assert np.array_equal(a, b)


def test_bf16_round_is_rne():
    x = np.array([1.0, 1.00390625, 1.01171875, -2.5e-3, 3.0e38], dtype=np.float32)
    r = synth.bf16_round(x)
    assert r[0] == 1.0 and r[1] == 1.0 and r[2] == np.float32(1.015625)
    assert np.all((r.view(np.uint32) & 0xFFFF) == 0)


def test_canonical_topk_tie_rule():
    s = np.array([[1.0, 3.0, 3.0, 2.0, 3.0]])
    val, idx = canonical_topk(s, 4)
    assert idx.tolist() == [[1, 2, 4, 3]]
    val, idx = canonical_topk(s, 7)
    assert idx[0, 5:].tolist() == [-1, -1] and np.isneginf(val[0, 5:]).all()


def test_exact_scores_cosine_formula(short_facts):
    q = short_facts[:3] * 2.0
    ex = exact_scores(short_facts, q, "cosine")
    assert np.allclose(np.diag(ex[:, :3]), 1.0, atol=1e-7) and ex.max() <= 1.0
