"""The screens' bound INPUTS: the per-row factors each screen reads, rows aligned with a
query's quantisation residual, rows and queries whose magnitudes overflow the bound's arithmetic. Every search must
equal the one-pass exact kernel (RR_KERNEL_EXACT) bit for bit — the contract of retriever.py:600-609 (the scores) and
:742-769 (the top-k) — and the cases are built so that the round-5 code returned a different top-1:

  * bf16 + dot: the int8 bound's eq |x| and eps terms read the row norms, which bf16 + dot storage never computed
    (they stayed at the 1.0 placeholder); a row of norm ~30 aligned with the query's one-piece residual then had a
    "bound" below its exact score, and 40 rows placed between the two kept it out of the verify's candidates while
    the verify proved a decoy;
  * bf16 + cosine: a row whose norm overflows fp32 (|x| > 1.8e19) has exact cosine 0, and a NaN bound, which the
    clip turned into -1: with every other row anti-correlated it is the true top-1 and the screen dropped it.

The per-row factors are also read back (rr_screen_factors) and compared with NumPy."""
import numpy as np
import pytest

from oracle import synth
from test_int8_bound import bf16_round, bound, quantize_query, quantize_rows, residual_aligned_row

pytestmark = pytest.mark.gpu

F = np.float32


@pytest.fixture
def Index(hip):
    from rag_service_amd import Index as _Index
    return _Index


def _same(a, b):
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0], equal_nan=True)


def _search_both(ix, q, k):
    """(the default path's results, the exact kernel's, screened blocks of the default path)"""
    ix.set_kernel("auto")
    got = ix.search(q, k)
    blocks = ix.screen_counts_all()[0]
    ix.set_kernel("exact")
    want = ix.search(q, k)
    ix.set_kernel("auto")
    return got, want, blocks


def _residual_trap(rng, n, d):
    """Query q0 (unit norm), and a corpus where row A = bf16(30 r^ + beta w) (residual_aligned_row: exact 0.5) is the
    top-1 for q0; a decoy D (exact eD, halfway between A's exact score and its unit-norm "bound" uA1) and 40 fillers
    whose bounds lie in (uA1, eD) — so with norms of 1 the verify's 32 candidates are D and 31 fillers, and it proves
    D. Background rows are small noise. Returns (corpus, q0, row of A, row of D)."""
    q0 = rng.standard_normal(d).astype(F)
    q0 /= np.linalg.norm(q0)
    qv = quantize_query(q0, 1)
    a = bf16_round(residual_aligned_row(q0, 30.0, target=0.5, pieces=1).astype(F)[None, :])

    def bounds(x, unit):
        xq, sx, e = quantize_rows(x)
        nd = np.sqrt((x * x).sum(axis=1, dtype=F)).astype(F)
        return bound(xq, sx, e, np.ones_like(nd) if unit else nd, *qv).astype(np.float64)

    e_a = float((a.astype(np.float64) @ q0.astype(np.float64))[0])
    u_a1 = float(bounds(a, True)[0])
    assert u_a1 < e_a - 0.08 and float(bounds(a, False)[0]) >= e_a      # the trap exists; the true bound holds
    e_d = 0.5 * (u_a1 + e_a)
    dec = bf16_round((e_d * q0)[None, :].astype(F))
    fill = bf16_round((np.linspace(u_a1 + 0.004, e_d - 0.014, 40)[:, None] * q0[None, :]).astype(F))
    fb = bounds(fill, False)
    assert fb.min() > u_a1 and fb.max() < e_d - 0.002, (fb.min(), fb.max(), u_a1, e_d)
    corpus = (rng.standard_normal((n, d)) * 0.003).astype(F)
    row_a, row_d = 1234, 5678
    corpus[row_a] = a[0]
    corpus[row_d] = dec[0]
    corpus[101 + 397 * np.arange(40)] = fill
    return corpus, q0, row_a, row_d


@pytest.mark.parametrize("b", [32, 64])
def test_bf16_dot_residual_aligned_row_is_found(Index, b):
    """bf16 + dot (the norms the int8 bound reads): every query slot holds q0, k = 1; the top-1 is
    row A, identical to the exact kernel. (32 query slots: the r6 32-slot bf16 screen; 64: the 64-slot one.)"""
    rng = np.random.default_rng(20261)
    n, d = 20000, 1024
    corpus, q0, row_a, _ = _residual_trap(rng, n, d)
    q = np.repeat(q0[None, :], b, axis=0)
    for metric in ("dot", "cosine"):
        ix = Index(dtype="bf16", metric=metric, options={"screen_i8_min_rows": 0})
        ix.load(corpus)
        assert ix.screen_int8()
        got, want, blocks = _search_both(ix, q, 1)
        assert blocks == 1
        _same(got, want)
        if metric == "dot":
            assert np.all(got[1][:, 0] == row_a)
        ix.close()


@pytest.mark.parametrize("scale,screened", [(2.0 ** 40, True), (2.0 ** 62, False), (2.0 ** 70, False)])
def test_bf16_cosine_huge_row_is_top1(Index, scale, screened):
    """One row scaled by 2^40 (norm 2^45: the screen's bound stays finite), 2^62 (norm above kBf16ScreenNorm = 2^60:
    the handle leaves the screen to the exact pass) or 2^70 (the fp32 norm overflows: exact cosine 0), aligned with
    query 0 while every other row is anti-correlated with it: it is query 0's top-1, identical to the exact kernel.
    (Round 5 kept screening the 2^70 row with a NaN bound clipped to -1 and returned a wrong top-1.)"""
    rng = np.random.default_rng(20262)
    n, d = 20000, 1024
    q = rng.standard_normal((32, d)).astype(F)
    q[0] /= np.linalg.norm(q[0])
    noise = rng.standard_normal((n, d)).astype(F) * F(0.3 / np.sqrt(d))
    corpus = (-q[0][None, :] + noise).astype(F)
    corpus[4321] = ((q[0] + noise[4321]) * scale).astype(F)
    ix = Index(dtype="bf16", metric="cosine", options={"screen_i8_min_rows": 0})
    ix.load(corpus)
    got, want, blocks = _search_both(ix, q, 5)
    assert blocks == (1 if screened else 0)
    _same(got, want)
    assert got[1][0, 0] == 4321
    ix.close()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("kind", ["huge", "nan"])
def test_huge_and_nan_queries_take_the_exact_pass(Index, dtype, kind):
    """A query with an element of 2^70 (|q| far beyond the screen's range: max|q| < 2^15) or a NaN element: the
    verify's range check flags the block, which is re-run exactly — results identical to the exact kernel's."""
    rng = np.random.default_rng(20263)
    n, d = 20000, 1024
    corpus = rng.standard_normal((n, d)).astype(F)
    q = rng.standard_normal((32, d)).astype(F)
    q[3, 17] = F(2.0 ** 70) if kind == "huge" else F(np.nan)
    for metric in ("dot", "cosine"):
        ix = Index(dtype=dtype, metric=metric, options={"screen_i8_min_rows": 0})
        ix.load(corpus)
        got, want, blocks = _search_both(ix, q, 5)
        assert blocks == 1
        _same(got, want)
        ix.close()


@pytest.mark.parametrize("dtype,metric", [("fp32", "dot"), ("fp32", "cosine"), ("bf16", "dot"), ("bf16", "cosine")])
def test_screen_factors_match_numpy(Index, dtype, metric):
    """The per-row factors the screens read (rr_screen_factors) against NumPy on the stored values: the row norm
    (fp32 sum of squares, any order: 1e-5 relative), the int8 scale max|x| / 127 (exact) and the error norm (an upper
    bound of |x - scale x8| within 1e-3 of it). bf16 + dot is the case round 5 left at 1.0. Rows of mixed scales, a
    zero row, a spiky row; then rows updated in place (rr_update_rows) are re-read."""
    rng = np.random.default_rng(20264)
    n, d = 70001, 1024
    x = rng.standard_normal((n, d)).astype(F) * rng.uniform(1e-3, 1e3, size=(n, 1)).astype(F)
    x[7] = 0
    x[8] *= F(0.01)
    x[8, 3] = F(500.0)
    ix = Index(dtype=dtype, metric=metric, options={"screen_i8_min_rows": 0})
    ix.load(x)

    def check(rows, ref):
        nrm, sc, er = ix.screen_factors(int(rows[0]), len(rows))
        v = bf16_round(ref) if dtype == "bf16" else ref
        want_n = np.sqrt((v.astype(np.float64) ** 2).sum(axis=1))
        assert np.allclose(nrm, want_n, rtol=1e-5, atol=0), float(np.max(np.abs(nrm - want_n) / np.maximum(want_n, 1e-30)))
        m = np.abs(v).max(axis=1)
        want_s = np.where(m > 0, m / F(127), F(0)).astype(F)
        assert np.array_equal(sc, want_s)
        with np.errstate(divide="ignore", invalid="ignore"):
            t = np.where(want_s[:, None] > 0, v / want_s[:, None], F(0)).astype(F)
        x8 = np.clip(np.rint(t), -127, 127)
        err = np.sqrt(((v.astype(np.float64) - want_s[:, None].astype(np.float64) * x8) ** 2).sum(axis=1))
        assert np.all(er.astype(np.float64) >= err), float(np.max(err - er))
        assert np.all(er.astype(np.float64) <= err * 1.001 + m.astype(np.float64) * np.sqrt(d) * 2.0 ** -21 + 1e-30)

    check(np.arange(0, 4096), x[:4096])
    check(np.arange(n - 513, n), x[n - 513:])
    idx = np.array([5, 4000, 70000])
    new = (rng.standard_normal((3, d)) * 37.0).astype(F)
    ix.update_rows(new, idx)
    for j, r in enumerate(idx):
        check(np.array([r]), new[j:j + 1])
    ix.close()


def test_exchange_with_two_buffer_sets(Index):
    """the exchange issue thread's lag follows the buffer sets in use (x_slots = 2 reuses block i -
    2's set, so block i waits until that exchange is issued). A 1-rank RCCL handle with two sets, many staged blocks
    and fetches in between: every result equals the exact kernel's."""
    from rag_service_amd import get_unique_id
    corpus = synth.unit_norm_gaussian(91, 70000, 1024)
    q = synth.unit_norm_gaussian(92, 32, 1024)
    ex = Index(dtype="fp32", metric="cosine")
    ex.load(corpus)
    ex.set_kernel("exact")
    want = ex.search(q, 5)
    ix = Index(dtype="fp32", metric="cosine", options={"x_slots": 2})
    ix.init_dist(1, 0, get_unique_id())
    ix.load(corpus)
    assert ix.get_option("x_slots") == 2
    ix.set_queries(q)
    for rnd in range(6):
        for _ in range(9):
            ix.search_staged(5)
        _same(ix.fetch(), want)
        _same(ix.search(q, 5), want)
    ix.close()
    ex.close()


def test_options_reject_unknown_and_out_of_range(Index):
    """rr_set_option: unknown names and values out of range are RR_E_INVALID; x_slots takes 2 or 4 only."""
    from rag_service_amd._lib import HipRetrievalError, RR_E_INVALID
    ix = Index(dtype="fp32", metric="dot")
    for name, value in (("no_such_option", 1), ("x_slots", 3), ("screen_ct8", 3), ("wide_verify", 2)):
        with pytest.raises(HipRetrievalError) as e:
            ix.set_option(name, value)
        assert e.value.code == RR_E_INVALID
    ix.set_option("screen_grid", 128)
    assert ix.get_option("screen_grid") == 128
    ix.close()


def test_update_rows_rejects_collectively(Index):
    """rr_update_rows under rr_init_dist is a collective: a rank whose arguments are invalid still reaches
    the ranks' agreement and fails with RR_E_INVALID (with a world of one, here, its own message); the handle stays
    usable — a valid update and a search follow, equal to the exact kernel on the updated corpus."""
    from rag_service_amd import get_unique_id
    from rag_service_amd._lib import HipRetrievalError, RR_E_INVALID
    corpus = synth.unit_norm_gaussian(93, 70000, 1024)
    q = synth.unit_norm_gaussian(94, 32, 1024)
    ix = Index(dtype="fp32", metric="cosine")
    ix.init_dist(1, 0, get_unique_id())
    ix.load(corpus)
    with pytest.raises(HipRetrievalError) as e:
        ix.update_rows(q[:2], np.array([5, 70000]))            # index out of range
    assert e.value.code == RR_E_INVALID and "outside" in str(e.value)
    with pytest.raises(HipRetrievalError) as e:
        ix.update_rows(q[:2, :512], np.array([5, 6]))          # wrong dimension
    assert e.value.code == RR_E_INVALID
    ix.update_rows(q[:2], np.array([5, 6]))
    corpus[[5, 6]] = q[:2]
    got = ix.search(q, 5)
    assert np.all(got[1][:2, 0] == [5, 6])
    ex = Index(dtype="fp32", metric="cosine")
    ex.load(corpus)
    ex.set_kernel("exact")
    _same(got, ex.search(q, 5))
    ex.close()
    ix.close()
