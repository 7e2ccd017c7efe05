"""Large k (32 < k <= 256) without sorting every key (rr_api.cpp large-k path): the split-K kernel keeps per
workgroup and query the top-k of its lane lists plus a floor, a radix select (select_kernel) picks the shard's
top-k and checks it against the floors, and an unproven block is re-run with the full sort. Results must be
BIT-IDENTICAL to the full-sort path (RR_KERNEL_EXACT) and match the oracle / the reference's goldens."""
import numpy as np
import pytest

from oracle import synth
from oracle.retriever_oracle import canonical_topk, exact_scores
from parity_helpers import check_topk

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Index(hip):
    from rag_service_amd import Index as _Index
    return _Index


def _same(got, want, msg=""):
    assert np.array_equal(got[1], want[1]), msg
    assert np.array_equal(got[0], want[0]), msg


CASES = [  # (n, d, b, k)
    (100, 1024, 32, 100), (1000, 1024, 32, 40), (5003, 512, 7, 64), (70001, 1024, 32, 100),
    (70001, 1024, 45, 256), (300000, 1024, 32, 33), (40, 256, 3, 64), (12345, 768, 1, 200),
]


@pytest.mark.parametrize("n,d,b,k", CASES)
@pytest.mark.parametrize("dtype,metric", [("fp32", "cosine"), ("fp32", "dot"), ("bf16", "cosine"),
                                          ("fp32-split", "dot")])
def test_large_k_equals_full_sort(Index, n, d, b, k, dtype, metric):
    if dtype == "bf16" and d % 512:
        pytest.skip("split-K bf16 needs d % 512 == 0 (the full sort serves it)")
    rng = np.random.default_rng(n + k + b)
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((b, d)).astype(np.float32)
    ix = Index(dtype=dtype, metric=metric)
    ix.load(corpus)
    got = ix.search(q, k)
    blocks, reruns = ix.screen_stats()
    assert blocks == -(-b // 32) and reruns == 0          # random data: every block proven complete
    ix.set_kernel("exact")
    want = ix.search(q, k)
    _same(got, want, (n, d, b, k))
    if dtype == "fp32" and n <= 70001:
        _, cidx = canonical_topk(exact_scores(corpus, q, metric), k)
        tol = 1e-3 * (np.sqrt(d) if metric == "dot" else 1.0)
        check_topk(got[1], got[0], cidx, corpus, q, metric, near_tie=1e-5 * np.sqrt(d), score_tol=tol)
    ix.close()


def _one_lane_rows(G, chunks_per_wg):
    """Rows that the static schedule hands to lane 0 of workgroup 0 for query slot 0..3's lane group: tile
    rows 0 and 1 (lane li takes rows 2li, 2li + 1) of both tiles of chunks 0, G, 2G, ... (64-row chunks)."""
    return np.array([c * G * 64 + t * 32 + e for c in range(chunks_per_wg) for t in (0, 1) for e in (0, 1)])


def test_large_k_unproven_block_is_rerun(Index):
    """Copies of one row placed exactly where one lane of one workgroup reads (more than its 32-entry list
    holds), queried with that row at k = 64: the lane drops copies that belong to the top-k, its floor says
    so, the block is flagged and re-run with the full sort — results equal the full sort's. Then the test
    hook forces the flag on every block."""
    import torch
    G = torch.cuda.get_device_properties(0).multi_processor_count   # the kernel's grid (one per CU)
    n = G * 64 * 20
    rows = _one_lane_rows(G, 20)                       # 80 rows in one lane list
    corpus = synth.unit_norm_gaussian(5, n, 1024)
    corpus[rows] = corpus[5]
    q = np.concatenate([corpus[5:6], synth.unit_norm_gaussian(6, 20, 1024)])
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    got = ix.search(q, 64)
    assert ix.screen_stats() == (1, 1)
    ix.set_kernel("exact")
    want = ix.search(q, 64)
    _same(got, want)
    assert list(got[1][0]) == sorted(np.append(rows, 5))[:64]   # ties in ascending index order
    ix.set_kernel("screen-fallback")
    _same(ix.search(q, 100), ix.set_kernel("exact") or ix.search(q, 100))
    ix.close()


@pytest.mark.parametrize("shards", [2, 8])
def test_large_k_sharded(Index, shards):
    rng = np.random.default_rng(shards + 100)
    corpus = rng.standard_normal((50000, 1024)).astype(np.float32)
    q = rng.standard_normal((40, 1024)).astype(np.float32)
    one = Index(dtype="fp32", metric="cosine")
    one.load(corpus)
    one.set_kernel("exact")
    many = Index(devices=[0] * shards, dtype="fp32", metric="cosine")
    many.load(corpus)
    for k in (33, 100, 256, 5, 64):
        _same(many.search(q, k), one.search(q, k), k)
    one.close()
    many.close()


def test_large_k_rccl_one_rank(Index):
    """The exchanged lists carry the shard's flag word after the keys; the final select reduces them, so a
    flagged shard makes the rank re-run."""
    import torch
    from rag_service_amd import get_unique_id
    G = torch.cuda.get_device_properties(0).multi_processor_count
    n = G * 64 * 20
    rows = _one_lane_rows(G, 20)
    corpus = synth.unit_norm_gaussian(3, n, 1024)
    corpus[rows] = corpus[9]
    q = np.concatenate([corpus[9:10], synth.unit_norm_gaussian(4, 31, 1024)])
    ref = Index(dtype="fp32", metric="dot")
    ref.load(corpus)
    ref.set_kernel("exact")
    rc = Index(dtype="fp32", metric="dot")
    rc.init_dist(1, 0, get_unique_id())
    rc.load(corpus)
    for k in (40, 256, 128):
        _same(rc.search(q, k), ref.search(q, k), k)
    assert rc.screen_stats() == (3, 3)                     # every block had the planted lane overflow
    ref.close()
    rc.close()


def test_large_k_async_and_staged(Index):
    rng = np.random.default_rng(8)
    corpus = rng.standard_normal((20000, 1024)).astype(np.float32)
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    ref = Index(dtype="fp32", metric="cosine")
    ref.load(corpus)
    ref.set_kernel("exact")
    qs = [rng.standard_normal((32, 1024)).astype(np.float32) for _ in range(4)]
    tickets = [ix.search_async(q, 100) for q in qs]
    for t, q in zip(tickets, qs):
        _same(ix.wait(t), ref.search(q, 100))
    ix.set_queries(qs[0])
    for _ in range(3):
        ix.search_staged(64)
    _same(ix.fetch(), ref.search(qs[0], 64))
    ix.close()
    ref.close()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
@pytest.mark.parametrize("dtype,metric", [("fp32", "cosine"), ("fp32", "dot"), ("bf16", "cosine")])
def test_full_key_path_k_above_256(Index, dtype, metric, devices):
    """k > 256: every key of the shard, then its top-k sorted by the hand-written select + sort (rr_topk.hip: radix
    select of the k-th key, compaction, bitonic 2048-key tiles, rank merges) — one tile, several tiles and merge
    passes, k = n (no select), k > n (zero padding -> -inf / -1) — and, with three shards, the serial exchange's
    merge of world x k candidates by the same routine. Against the oracle's canonical top-k (retriever.py:750-769),
    and bit-identical across shard counts. The largest k is the reference's own clamp k -> n (retriever.py:730)."""
    rng = np.random.default_rng(len(devices) * 7 + len(dtype) + len(metric))
    n, d, b = 20011, 256, 40
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    if dtype == "bf16":
        corpus = synth.bf16_round(corpus)
    q = rng.standard_normal((b, d)).astype(np.float32)
    ix = Index(devices=devices, dtype=dtype, metric=metric)
    ix.load(corpus)
    one = Index(dtype=dtype, metric=metric) if len(devices) > 1 else None
    if one:
        one.load(corpus)
    ex = exact_scores(corpus, q, metric)
    for k in (257, 2048, 2049, 7000, n, n + 9):
        scores, idx = ix.search(q, k)
        kk = min(k, n)
        _, cidx = canonical_topk(ex, kk)
        tol = 1e-3 * (np.sqrt(d) if metric == "dot" else 1.0)
        check_topk(idx[:, :kk], scores[:, :kk], cidx, corpus, q, metric, near_tie=1e-5 * np.sqrt(d), score_tol=tol)
        assert np.all(np.diff(scores[:, :kk], axis=1) <= 0), k
        if k > n:
            assert np.all(idx[:, n:] == -1) and np.all(np.isneginf(scores[:, n:])), k
        assert np.array_equal(np.sort(idx[:, :kk], axis=1), np.tile(np.arange(n), (b, 1))) if kk == n else True
        if one:
            _same(one.search(q, k), (scores, idx), k)
    ix.close()
    if one:
        one.close()
