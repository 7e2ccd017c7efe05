"""The bf16 storage's screened search (rr_sk.hip DT 9 + the DT 1 verify): the screen reads an int8 copy of the bf16 rows
(per-row scale and error norm, half the bf16 bytes) against ONE int8 piece per query — 64 query slots per pass, the
batch-64 configs' block — and the verify rescores the candidates with the bf16 pass's own arithmetic (the same K split,
MFMA order, wave order and epilogue), so results must be BIT-IDENTICAL to the one-pass bf16 kernel's. Blocks of <= 32
queries are screened in 32-slot blocks (r6; round 5 kept them on the exact 32-slot pass)."""
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


def _bf16(x):
    """fp32 -> the bf16 values (RNE) as fp32, the rows bf16 storage holds."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def _spiky_corpus(rng, n, d, q):
    """Random rows of mixed norms, a zero row, and rows built to be the queries' best matches while the int8 copy loses
    them (one large element sets the row's scale; only the error norm bounds the rest)."""
    corpus = rng.standard_normal((n, d)).astype(np.float32) * rng.uniform(0.25, 4, size=(n, 1)).astype(np.float32)
    corpus[n // 3] = 0.0
    rows = rng.choice(n, size=min(64, n // 2), replace=False)
    for j, r in enumerate(rows):
        v = q[j % len(q)] / np.linalg.norm(q[j % len(q)]) * 0.9 + 0.05 * rng.standard_normal(d).astype(np.float32)
        v[rng.integers(d)] = 60.0 * rng.choice([-1.0, 1.0])
        corpus[r] = v.astype(np.float32)
    return corpus


def _same(a, b):
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0], equal_nan=True)


@pytest.mark.parametrize("n,d,b,k", [(70001, 1024, 64, 10), (4099, 1024, 64, 5), (12345, 512, 40, 13),
                                     (65536, 1024, 33, 1), (257, 1024, 64, 4),
                                     # 32-slot blocks (r6): the headline batch, small batches, k up to 29 (32-entry lists)
                                     (70001, 1024, 32, 5), (12345, 512, 7, 16), (4099, 1024, 32, 29), (257, 1024, 1, 1)])
@pytest.mark.parametrize("metric", ["cosine", "dot"])
def test_bf16_screen_equals_exact(Index, n, d, b, k, metric):
    rng = np.random.default_rng(n + d + k + b)
    q = rng.standard_normal((b, d)).astype(np.float32)
    corpus = _spiky_corpus(rng, n, d, q)
    ix = Index(dtype="bf16", metric=metric)
    ix.load(corpus)
    assert ix.screen_int8() and ix.screen_copy()
    got = ix.search(q, k)
    blocks, flagged, reruns, _ = ix.screen_counts_all()
    assert blocks == 1 and reruns == flagged
    ix.set_kernel("exact")
    want = ix.search(q, k)
    _same(got, want)
    cb = _bf16(corpus)
    _, cidx = canonical_topk(exact_scores(cb, q, metric), k)
    tol = 1e-3 * (np.sqrt(d) * 4 if metric == "dot" else 1.0)
    check_topk(got[1], got[0], cidx, cb, q, metric, near_tie=1e-5 * np.sqrt(d) * 16, score_tol=tol)
    ix.close()


def test_bf16_screen_block_shapes(Index):
    """32 queries or fewer: one screened 32-slot block (r6); 33-64: one screened 64-slot block; 100: two 64-slot
    blocks; k = 20 (32-entry lists) at 32 queries: a 32-slot block too."""
    rng = np.random.default_rng(3)
    corpus = rng.standard_normal((20000, 1024)).astype(np.float32)
    ix = Index(dtype="bf16", metric="cosine")
    ix.load(corpus)
    q32 = rng.standard_normal((32, 1024)).astype(np.float32)
    got32 = ix.search(q32, 10)
    assert ix.screen_counts_all()[0] == 1
    ix.search(rng.standard_normal((64, 1024)).astype(np.float32), 10)
    assert ix.screen_counts_all()[0] == 2
    q = rng.standard_normal((100, 1024)).astype(np.float32)
    got = ix.search(q, 10)
    assert ix.screen_counts_all()[0] == 4
    got20 = ix.search(q32, 20)
    assert ix.screen_counts_all()[0] == 5
    ix.set_kernel("exact")
    _same(got32, ix.search(q32, 10))
    _same(got20, ix.search(q32, 20))
    ix.set_kernel("exact")
    _same(got, ix.search(q, 10))
    ix.close()


def test_bf16_screen_unit_norm_headline_shape(Index):
    """Config 5's data shape (unit-norm rows, B = 64, k = 10) on a 262144-row shard: no block re-runs, bit-identical."""
    corpus = synth.unit_norm_gaussian(1234, 262144, 1024)
    q = synth.unit_norm_gaussian(5678, 128, 1024)
    ix = Index(dtype="bf16", metric="cosine")
    ix.load(corpus)
    assert ix.screen_int8()
    got = ix.search(q, 10)
    blocks, flagged, reruns, _ = ix.screen_counts_all()
    assert (blocks, flagged, reruns) == (2, 0, 0)
    ix.set_kernel("exact")
    _same(got, ix.search(q, 10))
    ix.close()


def test_bf16_screen_forced_flags_rerun_exactly(Index):
    """The test hook flags every block (RR_KERNEL_SCREEN_FALLBACK): each is re-run by the exact pass."""
    rng = np.random.default_rng(7)
    corpus = rng.standard_normal((30000, 1024)).astype(np.float32)
    q = rng.standard_normal((64, 1024)).astype(np.float32)
    ix = Index(dtype="bf16", metric="dot")
    ix.load(corpus)
    ix.set_kernel("exact")
    want = ix.search(q, 8)
    ix.set_kernel("screen-fallback")
    got = ix.search(q, 8)
    blocks, flagged, reruns, _ = ix.screen_counts_all()
    assert blocks == 1 and flagged == 1 and reruns == 1
    _same(got, want)
    ix.close()


def test_bf16_clustered_corpus_goes_to_repair_mode(Index):
    """Contiguous near-duplicate clusters defeat the lists: flagged windows switch the handle to repair mode, where the
    verify marks the chunks to rescore and the repair pass (the bf16 64-slot kernel over those chunks) completes the
    slots in-stream; every search stays bit-identical to the exact pass."""
    rng = np.random.default_rng(11)
    n, d = 65536, 1024
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((64, d)).astype(np.float32)
    for j in range(64):   # 64 clusters of 40 near-copies of query j, contiguous
        base = q[j] / np.linalg.norm(q[j])
        r0 = 1000 * j
        corpus[r0:r0 + 40] = base + 0.002 * rng.standard_normal((40, d)).astype(np.float32)
    ix = Index(dtype="bf16", metric="cosine")
    ix.load(corpus)
    ix.set_kernel("exact")
    want = ix.search(q, 10)
    ix.set_kernel("auto")
    for _ in range(40):
        _same(ix.search(q, 10), want)
    full, _, _ = ix.screen_state()
    assert full
    assert ix.screen_repairs() > 0
    ix.close()


def test_bf16_update_rows_keeps_the_int8_copy(Index):
    """rr_update_rows re-quantises the updated rows' int8 copy (scale, error norm): the screen then finds rows moved
    next to the queries, and the index equals a fresh load of the updated corpus."""
    rng = np.random.default_rng(5)
    n, d = 40000, 1024
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((64, d)).astype(np.float32)
    ix = Index(dtype="bf16", metric="cosine")
    ix.load(corpus)
    idx = rng.choice(n, size=64, replace=False)
    new = (q + 0.01 * rng.standard_normal(q.shape)).astype(np.float32)
    ix.update_rows(new, idx)
    assert ix.screen_int8()
    got = ix.search(q, 10)
    assert ix.screen_counts_all()[0] == 1
    corpus[idx] = new
    ref = Index(dtype="bf16", metric="cosine")
    ref.load(corpus)
    ref.set_kernel("exact")
    _same(got, ref.search(q, 10))
    assert np.all(got[1][:, 0] == idx)
    ix.close()
    ref.close()


@pytest.mark.parametrize("bad", [np.inf, np.nan])
@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_non_finite_row_turns_the_screen_off(Index, bad, dtype):
    """A row with an infinite or NaN value has a non-finite error norm (bf16) or fails the f16 range (fp32): the bound
    cannot hold, so the handle does not screen (the exact pass serves it, results unchanged). (The range check's max
    counts a NaN as infinite: a plain fmaxf reduction drops NaNs.)"""
    rng = np.random.default_rng(9)
    corpus = rng.standard_normal((20000, 1024)).astype(np.float32)
    corpus[123, 5] = bad
    q = rng.standard_normal((64 if dtype == "bf16" else 32, 1024)).astype(np.float32)
    ix = Index(dtype=dtype, metric="dot")
    ix.load(corpus)
    got = ix.search(q, 10)
    assert ix.screen_counts_all()[0] == 0
    ix.set_kernel("exact")
    _same(got, ix.search(q, 10))
    ix.close()


@pytest.mark.parametrize("kind", ["tiny", "huge_row", "overflow_row"])
def test_bf16_screen_extreme_magnitudes(Index, kind):
    """Rows near bf16's range ends: tiny rows (2^-60 scale: squares underflow, the bound's absolute terms carry them),
    one huge row (2^40: norm 2^45, its bound stays finite) and one whose norm overflows fp32 (2^60 x a Gaussian row:
    |x| ~ 2^65 > kBf16ScreenNorm, so the handle leaves bf16 on the exact pass — round 5 screened it with a NaN bound
    clipped to -1; tests/test_gpu_bound_inputs.py makes that row the true top-1)."""
    rng = np.random.default_rng(13)
    n, d = 20000, 1024
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    if kind == "tiny":
        corpus *= np.float32(2.0 ** -60)
    else:
        corpus[777] *= np.float32(2.0 ** (40 if kind == "huge_row" else 60))
    q = rng.standard_normal((64, d)).astype(np.float32)
    for metric in ("dot", "cosine"):
        ix = Index(dtype="bf16", metric=metric)
        ix.load(corpus)
        got = ix.search(q, 10)
        assert ix.screen_counts_all()[0] == (0 if kind == "overflow_row" else 1)
        ix.set_kernel("exact")
        _same(got, ix.search(q, 10))
        ix.close()
