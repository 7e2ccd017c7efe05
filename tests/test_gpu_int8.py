"""The int8 screen (rr_sk.hip DT 8, fp32 storage with d a multiple of 512 up to 1024): the screened search's upper
bounds from an int8 copy of the rows (per-row scale and error norm) against two int8 pieces of each query. Its bound
is looser than the f16 copy's, so more rows reach the verify (its wide phase takes every list entry whose bound
reaches the exact k-th score); results must stay BIT-IDENTICAL to the one-pass exact kernel, including on rows the
int8 copy represents badly (one large element: the rest rounds to zero and only the error norm bounds the score)."""
import numpy as np
import pytest

from oracle import synth
from oracle.retriever_oracle import canonical_topk, exact_scores
from parity_helpers import check_topk

pytestmark = pytest.mark.gpu


@pytest.fixture
def Index(hip, monkeypatch):
    """(the int8 copy is made for shards of any size here: RR_SCREEN_I8_MIN_ROWS=0)"""
    from rag_service_amd import Index as _Index
    monkeypatch.setenv("RR_SCREEN_I8_MIN_ROWS", "0")
    return _Index


def _spiky_corpus(rng, n, d, q):
    """Random rows of mixed norms, a zero row, and 64 rows built to be the queries' best matches while the int8 copy
    loses them: a large spike in one element sets the row's scale, so the part aligned with the query rounds to 0."""
    corpus = rng.standard_normal((n, d)).astype(np.float32) * rng.uniform(0.25, 4, size=(n, 1)).astype(np.float32)
    corpus[n // 3] = 0.0
    rows = rng.choice(n, size=min(64, n // 2), replace=False)
    for j, r in enumerate(rows):
        v = q[j % len(q)] / np.linalg.norm(q[j % len(q)]) * 0.9 + 0.05 * rng.standard_normal(d).astype(np.float32)
        v[rng.integers(d)] = 60.0 * rng.choice([-1.0, 1.0])   # 60 >> the rest: sx ~ 0.47, every other element -> 0
        corpus[r] = v.astype(np.float32)
    return corpus


@pytest.mark.parametrize("pieces", ["2", "1"])
@pytest.mark.parametrize("n,d,b,k", [(4099, 1024, 32, 5), (70001, 1024, 32, 10), (65536, 512, 20, 1),
                                     (12345, 1024, 7, 16), (33, 1024, 32, 3)])
@pytest.mark.parametrize("metric", ["cosine", "dot"])
def test_int8_screen_equals_exact(Index, monkeypatch, n, d, b, k, metric, pieces):
    """(pieces "1": the one-query-piece form, DT 9 at 32 slots, which large shards screen with — forced here at every
    size, option screen_i8_pieces)"""
    rng = np.random.default_rng(n + d + k)
    q = rng.standard_normal((b, d)).astype(np.float32)
    corpus = _spiky_corpus(rng, n, d, q)
    ix = Index(dtype="fp32", metric=metric, options={"screen_i8_pieces": int(pieces)})
    ix.load(corpus)
    assert ix.screen_int8()
    got = ix.search(q, k)
    blocks, flagged, reruns, _ = ix.screen_counts_all()
    assert blocks == 1 and reruns == flagged
    ix.set_kernel("exact")
    want = ix.search(q, k)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    ix.set_kernel("auto")
    ix.screen_int8(False)
    assert not ix.screen_int8()
    f16 = ix.search(q, k)
    assert np.array_equal(f16[1], want[1]) and np.array_equal(f16[0], want[0])
    _, cidx = canonical_topk(exact_scores(corpus, q, metric), k)
    tol = 1e-3 * (np.sqrt(d) * 4 if metric == "dot" else 1.0)
    check_topk(got[1], got[0], cidx, corpus, q, metric, near_tie=1e-5 * np.sqrt(d) * 16, score_tol=tol)
    ix.close()


def test_int8_screen_proves_unit_norm_blocks(Index):
    """The headline's data: with 16-entry lists the int8 bound leaves more than KT - k candidates above the exact
    k-th score for many queries. The verify's first tile rescores the top 32 bounds (r5; 16 before, when ~40 % of the
    slots needed the wide phase — entries whose bound reaches the exact k-th — for 1-2 more tiles): no block re-runs,
    the wide phase takes at most a few slots, and the results equal the exact kernel's."""
    corpus = synth.unit_norm_gaussian(1234, 262144, 1024)
    q = synth.unit_norm_gaussian(5678, 128, 1024)
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    assert ix.screen_int8()
    got = ix.search(q, 5)
    blocks, flagged, reruns, wide = ix.screen_counts_all()
    assert (blocks, flagged, reruns) == (4, 0, 0)
    assert wide <= 16   # (r4, 16 candidates: ~50 of the 128 slots)
    ix.set_kernel("exact")
    want = ix.search(q, 5)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    ix.close()


def test_int8_screen_forced_reruns_then_pause(Index):
    """Adaptive (r5): a window of settled blocks that re-ran (forced here: RR_KERNEL_SCREEN_FALLBACK flags every block)
    switches the handle to repair mode, keeping the int8 copy; forced flags go on (the test hook bypasses the repair),
    so the next window pauses screening; results stay exact throughout; a reload re-arms everything."""
    rng = np.random.default_rng(3)
    corpus = rng.standard_normal((20000, 1024)).astype(np.float32)
    q = rng.standard_normal((32, 1024)).astype(np.float32)
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    ix.set_kernel("exact")
    want = ix.search(q, 5)
    ix.set_kernel("screen-fallback")
    assert ix.screen_int8()
    for _ in range(32):
        got = ix.search(q, 5)
        assert np.array_equal(got[1], want[1])
    assert ix.screen_int8() and ix.screen_state() == (True, 0, 0)     # repair mode, the int8 copy still screening
    for _ in range(32):
        got = ix.search(q, 5)
        assert np.array_equal(got[1], want[1])
    assert ix.screen_state() == (True, 1024, 1)                       # still flagging in repair mode: paused
    ix.set_kernel("auto")
    got = ix.search(q, 5)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    ix.load(corpus)
    assert ix.screen_int8() and ix.screen_state() == (False, 0, 0)
    ix.close()


def test_int8_screen_sharded_and_odd_rows(Index):
    """Shards of odd row counts (the int8 copy's padding row) in one process, exchange path: identical to exact."""
    rng = np.random.default_rng(11)
    n, d = 30001, 1024
    q = rng.standard_normal((32, d)).astype(np.float32)
    corpus = _spiky_corpus(rng, n, d, q)
    ix = Index(dtype="fp32", metric="cosine", devices=[0, 0, 0])
    ix.load(corpus)
    assert ix.screen_int8()
    got = ix.search(q, 8)
    ix.set_kernel("exact")
    want = ix.search(q, 8)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    ix.close()


@pytest.mark.parametrize("ct", ["2", "4"])
def test_int8_screen_chunk_sizes(Index, monkeypatch, ct):
    """The int8 screen's dynamic-schedule chunk (2 tiles of 64 rows below 500k rows per shard, else 4; option
    screen_ct8 forces either): any chunk size gives the exact kernel's results, on the static schedule too."""
    rng = np.random.default_rng(int(ct))
    n, d = 150001, 1024
    q = rng.standard_normal((32, d)).astype(np.float32)
    corpus = _spiky_corpus(rng, n, d, q)
    ix = Index(dtype="fp32", metric="cosine", options={"screen_ct8": int(ct)})
    ix.load(corpus)
    assert ix.screen_int8()
    got = [ix.search(q, 5)]
    ix.set_schedule(False)
    got.append(ix.search(q, 5))
    ix.set_kernel("exact")
    want = ix.search(q, 5)
    for g in got:
        assert np.array_equal(g[1], want[1]) and np.array_equal(g[0], want[0])
    ix.close()
