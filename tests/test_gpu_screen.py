"""The screened search (fp32 storage, rr_sk.hip "Screened search"): an f16 screening pass of upper bounds,
exact rescoring of the KT candidates with the DT 3 arithmetic, and an exact fallback pass when the bound cannot
prove completeness. Its results must be BIT-IDENTICAL to the one-pass exact kernel (RR_KERNEL_EXACT) in every
case — screened, forced fallback, shards, cosine and dot — and match the oracle."""
import functools

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


CASES = [  # (n, d, b, k)
    (1, 256, 1, 1), (5, 256, 3, 5), (40, 1024, 32, 29), (1000, 512, 32, 8), (4099, 1024, 32, 5),
    (12345, 1024, 20, 16), (2049, 768, 7, 2), (70000, 1024, 32, 10), (33, 256, 45, 3),
]


@pytest.mark.parametrize("n,d,b,k", CASES)
@pytest.mark.parametrize("metric", ["cosine", "dot"])
def test_screened_equals_exact(Index, n, d, b, k, metric):
    rng = np.random.default_rng(n + d + b + k)
    corpus = rng.standard_normal((n, d)).astype(np.float32) * rng.uniform(0.5, 2, size=(n, 1)).astype(np.float32)
    q = rng.standard_normal((b, d)).astype(np.float32)
    ix = Index(dtype="fp32", metric=metric)
    ix.load(corpus)
    got = ix.search(q, k)
    blocks, fallbacks = ix.screen_stats()
    assert blocks == -(-b // 32)
    ix.set_kernel("exact")
    want = ix.search(q, k)
    ix.set_kernel("screen-fallback")
    forced = ix.search(q, k)
    assert ix.screen_stats()[1] == fallbacks + blocks          # every forced block took the exact pass
    for s, i in (got, forced):
        assert np.array_equal(i, want[1]) and np.array_equal(s, want[0])
    _, cidx = canonical_topk(exact_scores(corpus, q, metric), k)
    tol = 1e-3 * (np.sqrt(d) if metric == "dot" else 1.0)
    check_topk(got[1], got[0], cidx, corpus, q, metric, near_tie=1e-5 * np.sqrt(d), score_tol=tol)
    ix.close()


def test_screen_rarely_falls_back_on_unit_norm_data(Index):
    """The headline's data (unit-norm rows): with a list of 2k + 2 the bound proves completeness for every
    block (at k near the list width, 29 of 32, a block may need the exact pass; the results are exact
    either way)."""
    corpus = synth.unit_norm_gaussian(1234, 65536, 1024)
    q = synth.unit_norm_gaussian(5678, 32, 1024)
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    for k in (1, 5, 10, 15):
        ix.search(q, k)
    assert ix.screen_stats() == (4, 0)
    ix.set_kernel("exact")
    want = ix.search(q, 29)
    ix.set_kernel("auto")
    got = ix.search(q, 29)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    ix.close()


@pytest.mark.parametrize("i8", [True, False])
@pytest.mark.parametrize("wide", [True, False])
def test_screen_ties_take_the_exact_pass(Index, monkeypatch, wide, i8):
    """40 copies of one row spread over the corpus, queried with that row: 40 exactly tied top scores, more
    than the screen's global candidate list holds. The verify's wide phase rescores every list entry above the
    largest single-list bound (the copies lie in many workgroups' lists) and proves the top-k; without it
    (option wide_verify = 0) the bound cannot prove completeness and the search is re-run exactly. Either way the
    result is the canonical order (equal scores by ascending index), bit-identical to the one-pass exact kernel,
    for cosine and dot."""
    corpus = synth.unit_norm_gaussian(77, 65536, 1024)
    dup = np.arange(40) * 1601 + 7
    corpus[dup] = corpus[123]
    q = np.concatenate([corpus[123:124], synth.unit_norm_gaussian(78, 31, 1024)])
    for metric in ("cosine", "dot"):
        ix = Index(dtype="fp32", metric=metric, options={"wide_verify": 1 if wide else 0})
        ix.load(corpus)
        assert ix.screen_int8() and ix.screen_int8(i8) == i8
        got = ix.search(q, 5)
        blocks, flagged, reruns, wide_slots = ix.screen_counts_all()
        if i8:   # (the int8 bound also sends other query slots through the wide phase)
            assert (blocks, flagged, reruns) == ((1, 0, 0) if wide else (1, 1, 1)) and (wide_slots >= 1) == wide
        else:
            assert (blocks, flagged, reruns, wide_slots) == ((1, 0, 0, 1) if wide else (1, 1, 1, 0))
        assert sorted(got[1][0]) == sorted(np.sort(np.append(dup, 123))[:5])
        ix.set_kernel("exact")
        want = ix.search(q, 5)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
        val, cidx = canonical_topk(exact_scores(corpus, q, metric), 5)
        assert np.array_equal(got[1], cidx)
        ix.close()


def test_screen_guards_f16_range(Index):
    """Values the screen's f16 reading cannot hold: a corpus element >= 2^15 turns screening off for the
    handle; a query element >= 2^15 makes its block take the exact pass. Both still give exact results."""
    rng = np.random.default_rng(9)
    corpus = rng.standard_normal((3000, 256)).astype(np.float32)
    q = rng.standard_normal((8, 256)).astype(np.float32)
    q[3, 17] = 40000.0
    ix = Index(dtype="fp32", metric="dot")
    ix.load(corpus)
    got = ix.search(q, 6)
    assert ix.screen_stats() == (1, 1)
    ix.set_kernel("exact")
    want = ix.search(q, 6)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    big = corpus.copy()
    big[5, 3] = 1e5
    ix.set_kernel("auto")
    ix.load(big)
    ix.search(q[:2], 4)
    assert ix.screen_stats() == (0, 0)                          # counters restart at the load; nothing screened
    ix.close()


@functools.lru_cache(maxsize=None)
def _tiny_cases():
    """Corpora and queries with elements in and below the f16 subnormal range (|x| < 2^-14 = 6.1e-5): there the
    screen's f16 values keep only a few significant bits (or round to 0), and its bound leans on the absolute
    rounding term eps_b (<= 2^-25 per element, rr_api.cpp kScreenEpsB) — valid only if neither the conversions nor
    the f16 MFMA flush subnormal inputs. Each case: (name, corpus, queries)."""
    rng = np.random.default_rng(2024)
    n, d, b = 20011, 1024, 32
    base = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((b, d)).astype(np.float32)
    cases = []
    for e in (14, 18, 22):                                     # every row scaled into / below the subnormal range
        cases.append((f"rows_2^-{e}", base * np.float32(2.0 ** -e), q))
    cases.append(("queries_2^-16", base, q * np.float32(2.0 ** -16)))
    cases.append(("both_2^-12", base * np.float32(2.0 ** -12), q * np.float32(2.0 ** -12)))
    mixed = base * np.exp2(-rng.integers(0, 25, size=(n, 1))).astype(np.float32)   # 2^0 .. 2^-24 per row
    cases.append(("mixed_scales", mixed, q))
    # the top rows are tiny: near-copies of each query scaled by 2^-20 (cosine ranks them first; by dot they sit
    # among rows of scale 2^-10), plus full-scale rows anti-aligned with the queries
    top = base * np.float32(2.0 ** -10)
    for i in range(b):
        for j in range(3):
            near = q[i] + 0.05 * rng.standard_normal(d).astype(np.float32)
            top[97 + 613 * i + 5 * j] = near * np.float32(2.0 ** -20)
    big = rng.choice(n, 300, replace=False)
    big = big[(big - 97) % 613 >= 16]
    top[big] = -q[rng.integers(0, b, big.size)] * np.float32(4.0)
    cases.append(("tiny_top_rows", top, q))
    # rows AND queries tiny together: the int8 screen's scale product sx * q8sc and its estimate
    # fall into fp32's subnormal range, the exact kernel's smaller split products below fp32's normal range
    cases.append(("both_2^-60", (base.astype(np.float64) * 2.0 ** -60).astype(np.float32),
                  (q.astype(np.float64) * 2.0 ** -60).astype(np.float32)))
    return cases


@pytest.mark.parametrize("i8", [False, True])
@pytest.mark.parametrize("case", range(8))
@pytest.mark.parametrize("metric", ["cosine", "dot"])
def test_screen_subnormal_range(Index, monkeypatch, case, metric, i8):
    """f16-subnormal magnitudes: rows scaled by 2^-14 / 2^-18 / 2^-22, tiny queries, mixed
    per-row scales, tiny top rows, and rows and queries both at 2^-60. Through the int8 copy (i8: the copy made for
    this 20011-row corpus, RR_SCREEN_I8_MIN_ROWS=0), the f16 copy, and the fp32-reading screen,
    the screened search must return results BIT-IDENTICAL to the one-pass exact kernel, and the oracle's top-k (fp64
    scores; index swaps only between numerically tied documents, relative to the scores' own scale)."""
    name, corpus, q = _tiny_cases()[case]
    ex = Index(dtype="fp32", metric=metric)
    ex.load(corpus)
    ex.set_kernel("exact")
    if i8:
        monkeypatch.setenv("RR_SCREEN_I8_MIN_ROWS", "0")
    ix = Index(dtype="fp32", metric=metric)
    monkeypatch.delenv("RR_SCREEN_I8_MIN_ROWS", raising=False)
    ix.load(corpus)
    assert ix.screen_copy()
    assert ix.screen_int8() == i8
    exact = exact_scores(corpus, q, metric)
    for k in (1, 5, 10):
        want = ex.search(q, k)
        got16 = ix.search(q, k)
        assert np.array_equal(got16[1], want[1]) and np.array_equal(got16[0], want[0]), (name, k)
        _, cidx = canonical_topk(exact, k)
        scale = float(np.max(np.abs(np.take_along_axis(exact, cidx, axis=1))))
        if name == "both_2^-60":   # (the exact kernel's own rounding of its sub-normal-range split products)
            check_topk(got16[1], got16[0], cidx, corpus, q, metric, near_tie=1e-3 * scale + 1e-300,
                       score_tol=1e-3 * max(scale, 1e-300) if metric == "dot" else 1e-3)
        else:
            check_topk(got16[1], got16[0], cidx, corpus, q, metric, near_tie=2e-5 * scale + 1e-30,
                       score_tol=1e-3 * max(scale, 1e-30) if metric == "dot" else 1e-3)
    blocks16, flagged16 = ix.screen_stats()
    ix.screen_copy(False)                                      # DT 6: the fp32 rows rounded to f16 in registers
    for k in (1, 5, 10):
        want = ex.search(q, k)
        got32 = ix.search(q, k)
        assert np.array_equal(got32[1], want[1]) and np.array_equal(got32[0], want[0]), (name, k)
    blocks, flagged = ix.screen_stats()
    assert blocks == 6 and blocks16 == 3
    print(f"{name} {metric}: flagged {flagged16}/3 ({'int8' if i8 else 'f16'} copy), "
          f"{flagged - flagged16}/3 (fp32 screen)")
    ix.close()
    ex.close()


def test_screen_f16_conversion_keeps_subnormals(Index):
    """The property the bound relies on, observed directly: the screen's bound stays valid only if f16 subnormal
    values are neither flushed by the conversion nor by the MFMA. A corpus of one-hot rows whose single non-zero
    element is an f16 subnormal (k * 2^-24, k = 1..1023), each queried by the matching one-hot query of a large
    value, makes the f16 product the ONLY non-zero term of every score. Kept, the screen's top-4 for query c are
    column c's rows and the exact top-1 (>= 513 * 2^-14) clears the 4th bound (~1.5e-4): no block flagged. Flushed,
    every u would be the bound's |x|-proportional terms alone, the top-4 would be rows 1019-1022 for every query,
    their exact scores 0, and the block flagged. Dot, k = 1: results bit-identical to the exact kernel, 0 flagged."""
    d = 512                                                    # the f16 copy serves d % 512 == 0
    n = 1023
    corpus = np.zeros((n, d), dtype=np.float32)
    col = np.arange(n) % d
    corpus[np.arange(n), col] = (np.arange(n) + 1).astype(np.float32) * np.float32(2.0 ** -24)
    q = np.zeros((d, d), dtype=np.float32)
    q[np.arange(d), np.arange(d)] = 1024.0
    ex = Index(dtype="fp32", metric="dot")
    ex.load(corpus)
    ex.set_kernel("exact")
    ix = Index(dtype="fp32", metric="dot")
    ix.load(corpus)
    want = ex.search(q[:32], 1)
    got = ix.search(q[:32], 1)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    # query column c: rows c and c + 512 (if < 1023): the last one holds the largest value
    expect = np.array([max(r for r in range(c, n, d)) for c in range(32)])
    assert np.array_equal(got[1][:, 0], expect)
    assert ix.screen_stats() == (1, 0)                         # proven by the screen: subnormals were kept
    ix.screen_copy(False)                                      # the same through the fp32-reading screen (DT 6)
    got = ix.search(q[:32], 1)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    assert ix.screen_stats() == (2, 0)
    ix.close()
    ex.close()


def _clustered(n, sigma, layout, seed=20260, clusters=1000):
    """n rows from the reference's real e5 rows (the first `clusters` of data/squad_embeddings.npy) plus seeded
    noise of relative size sigma, L2-normalised: 'interleaved' (row i from SQuAD row i mod clusters) or
    'contiguous' (row i from SQuAD row i div (n / clusters))."""
    import os
    sq = np.load(os.path.join(os.path.dirname(__file__), "golden", "data", "squad_embeddings.npy")).astype(np.float32)
    sq = sq[:clusters] / np.linalg.norm(sq[:clusters], axis=1, keepdims=True)
    rng = np.random.default_rng(seed)
    m = clusters
    c = np.arange(n) % m if layout == "interleaved" else np.minimum(np.arange(n) // (n // m), m - 1)
    x = sq[c] + np.float32(sigma) * rng.standard_normal((n, sq.shape[1]), dtype=np.float32) / np.float32(32.0)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    qc = rng.integers(0, m, 32)
    q = sq[qc] + np.float32(sigma) * rng.standard_normal((32, sq.shape[1]), dtype=np.float32) / np.float32(32.0)
    return x, q / np.linalg.norm(q, axis=1, keepdims=True)


@pytest.mark.parametrize("metric", ["cosine", "dot"])
@pytest.mark.parametrize("layout", ["interleaved", "contiguous"])
def test_wide_verify_on_clustered_embeddings(Index, metric, layout):
    """Near-duplicate clusters: 60 noisy copies (sigma 0.01) of each of the 1000 real SQuAD e5
    rows. Far more than 16 documents lie inside the screen's bound window above each query's k-th score, so the
    first check fails for every query. Interleaved, each workgroup's list holds its few copies and the wide phase
    proves the top-k on the device (no flag, no re-run); contiguous, a cluster fills a few workgroups' lists and
    the block takes the exact pass. Results bit-identical to the exact kernel either way, for k = 5 and 10."""
    corpus, q = _clustered(60000, 0.01, layout)
    ex = Index(dtype="fp32", metric=metric)
    ex.load(corpus)
    ex.set_kernel("exact")
    ix = Index(dtype="fp32", metric=metric)
    ix.load(corpus)
    for k in (5, 10):
        want = ex.search(q, k)
        got = ix.search(q, k)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), k
    blocks, flagged, reruns, wide_slots = ix.screen_counts_all()
    print(layout, metric, {"blocks": blocks, "flagged": flagged, "reruns": reruns, "wide_slots": wide_slots})
    assert blocks == 2
    if layout == "interleaved":
        assert flagged == 0 and reruns == 0 and wide_slots >= 32
    else:
        assert flagged == reruns and flagged >= 1
    ix.close()
    ex.close()


def _plain_and_dist(Index, corpus):
    """The same corpus in a plain handle and in one with a 1-rank RCCL communicator (rr_init_dist: every search takes
    the multi-process data path — all-gather of the candidates with the flag words, device merge). Both on the static
    chunk schedule: the dynamic one hands rows to workgroups by a race, so which blocks a clustered corpus flags
    varies from run to run (the results never do); static, the screen's lists and so the flags are reproducible, and
    the two handles must then switch at the same searches."""
    from rag_service_amd import get_unique_id
    plain = Index(dtype="fp32", metric="cosine")
    plain.load(corpus)
    dist = Index(dtype="fp32", metric="cosine")
    dist.init_dist(1, 0, get_unique_id())
    dist.load(corpus)
    for ix in (plain, dist):
        ix.set_schedule(False)
    return plain, dist


@pytest.mark.parametrize("layout", ["interleaved", "contiguous"])
def test_screen_adapts_to_clustered_corpora(Index, layout):
    """The adaptive screen (rr_api.cpp observe_settled) on 1000 noisy copies of each of 100 SQuAD rows (sigma 0.01):
    interleaved, every cluster's copies fall on a few lanes of each workgroup (a stride of 100 rows) and the wide
    phase, barred at the exact k-th score, proves every block with the short lists and the int8 copy (no flags, no
    switch). Contiguous, a cluster fills a few workgroups' lists: after a window of re-run blocks the handle switches
    to repair mode (r5: full lists + per-chunk maxima, the unproven slots' chunks rescored exactly in-stream) and no
    block flags after that, the int8 copy screening throughout. Decided from settled searches only, so a handle in
    multi-process mode (1-rank RCCL communicator) switches at exactly the same searches as a plain one. Results
    bit-identical to the exact kernel at every step."""
    corpus, q = _clustered(100000, 0.01, layout, clusters=100)
    ex = Index(dtype="fp32", metric="cosine")
    ex.load(corpus)
    ex.set_kernel("exact")
    want = ex.search(q, 5)
    handles = _plain_and_dist(Index, corpus)
    hists = []
    for ix in handles:
        assert ix.screen_state() == (False, 0, 0)
        hist = []
        for step in range(100):
            got = ix.search(q, 5)
            assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), step
            hist.append(ix.screen_counts_all() + ix.screen_state() + (ix.screen_int8(),))
        hists.append(hist)
        ix.close()
    hist, hist_dist = hists
    assert [h[4:] for h in hist] == [h[4:] for h in hist_dist]          # the same switch points, step by step
    assert [h[:3] for h in hist] == [h[:3] for h in hist_dist]          # the same blocks, flags and re-runs
    blocks, flagged, reruns, wide_slots, full, pause_left, pauses, i8 = hist[-1]
    print(layout, hist[40], hist[-1])
    assert all(h[7] for h in hist)                                      # the int8 copy screens throughout
    if layout == "interleaved":
        # r4: the wide phase bars at the exact k-th score once that clears the lists' tail, so the short lists prove
        # every block of the interleaved clusters (r3 needed a window of re-runs and the full lists first)
        assert flagged == 0 and pauses == 0 and not full and blocks == 100 and wide_slots >= 32 * 100
    else:
        # repair mode at the end of the first window; no flag, re-run or pause after it
        full_at = next(i for i, h in enumerate(hist) if h[4])
        assert full_at == 31 and pauses == 0 and blocks == 100
        assert flagged == hist[full_at][1] and reruns == hist[full_at][2]
    ex.close()


@pytest.mark.parametrize("shards", [2, 8])
def test_screened_sharded_equals_single(Index, shards):
    """Shards screen and verify independently (each with its own fallback decision) before the exchange:
    results equal the one-shard exact ones, for the pipelined (staged) loop too."""
    rng = np.random.default_rng(shards)
    corpus = rng.standard_normal((20011, 1024)).astype(np.float32)
    corpus /= np.linalg.norm(corpus, axis=1, keepdims=True)
    q = rng.standard_normal((45, 1024)).astype(np.float32)
    one = Index(devices=[0], dtype="fp32", metric="cosine")
    one.load(corpus)
    one.set_kernel("exact")
    many = Index(devices=[0] * shards, dtype="fp32", metric="cosine")
    many.load(corpus)
    for k in (5, 10, 29, 40):
        want = one.search(q, k)
        got = many.search(q, k)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), k
    many.set_queries(q)
    for _ in range(5):
        many.search_staged(5)
    s, i = many.fetch()
    want = one.search(q, 5)
    assert np.array_equal(i, want[1]) and np.array_equal(s, want[0])
    many.set_kernel("screen-fallback")
    got = many.search(q, 7)
    want = one.search(q, 7)
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    one.close()
    many.close()


def test_screened_rccl_one_rank(Index):
    from rag_service_amd import get_unique_id
    rng = np.random.default_rng(12)
    corpus = rng.standard_normal((9000, 512)).astype(np.float32)
    q = rng.standard_normal((32, 512)).astype(np.float32)
    ref = Index(dtype="fp32", metric="cosine")
    ref.load(corpus)
    ref.set_kernel("exact")
    rc = Index(dtype="fp32", metric="cosine")
    rc.init_dist(1, 0, get_unique_id())
    rc.load(corpus)
    for k in (3, 12):
        want = ref.search(q, k)
        got = rc.search(q, k)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), k
    ref.close()
    rc.close()


@pytest.mark.parametrize("metric", ["cosine", "dot"])
def test_dynamic_schedule_equals_static(Index, metric):
    """The screen's dynamic chunk schedule (9th wave dequeuing chunks from a device counter that each launch
    resets) against the static round-robin one: identical results over back-to-back launches of different
    sizes on one handle (a counter left wrong by one launch would skip or repeat chunks in the next)."""
    rng = np.random.default_rng(31)
    corpus = rng.standard_normal((70001, 1024)).astype(np.float32)
    corpus /= np.linalg.norm(corpus, axis=1, keepdims=True)
    ix = Index(dtype="fp32", metric=metric)
    ix.load(corpus)
    st = Index(dtype="fp32", metric=metric)
    st.load(corpus)
    st.set_schedule(False)
    for b, k in [(32, 5), (7, 1), (32, 7), (45, 3), (1, 5)] * 3:
        q = rng.standard_normal((b, 1024)).astype(np.float32)
        got = ix.search(q, k)
        want = st.search(q, k)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), (b, k)
    ix.set_queries(q)
    for _ in range(50):
        ix.search_staged(5)
    s, i = ix.fetch()
    want = st.search(q, 5)
    assert np.array_equal(i, want[1]) and np.array_equal(s, want[0])
    small = Index(dtype="fp32", metric=metric)       # fewer chunks than workgroups, and a single chunk
    for n in (1000, 40, 257 * 64):
        small.load(corpus[:n])
        st.load(corpus[:n])
        got = small.search(q, 5)
        want = st.search(q, 5)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), n
    ix.close()
    st.close()
    small.close()


@pytest.mark.parametrize("metric", ["cosine", "dot"])
def test_screen_copy_equals_fp32_screen_and_exact(Index, metric):
    """The screen over the f16 copy (DT 7, half the bytes) and the screen over the fp32 rows (DT 6) both
    end in the exact fp32 verify: results bit-identical to each other and to the one-pass exact kernel,
    across reloads and with the copy freed."""
    rng = np.random.default_rng(77)
    corpus = rng.standard_normal((20011, 1024)).astype(np.float32) * rng.uniform(0.5, 2, (20011, 1)).astype(np.float32)
    q = rng.standard_normal((45, 1024)).astype(np.float32)
    ix = Index(dtype="fp32", metric=metric)
    ix.load(corpus)
    assert ix.screen_copy()                                   # made at load (default)
    ex = Index(dtype="fp32", metric=metric)
    ex.load(corpus)
    ex.set_kernel("exact")
    for k in (1, 5, 10, 29):
        want = ex.search(q, k)
        got16 = ix.search(q, k)
        ix.screen_copy(False)
        assert not ix.screen_copy()
        got32 = ix.search(q, k)
        for got in (got16, got32):
            assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), k
        ix.screen_copy(True)
        ix.load(corpus)                                       # the copy comes back with the next load
        assert ix.screen_copy()
    ix.close()
    ex.close()


def test_narrow_lists_then_repair_mode(Index):
    """k = 10 screens with 16-entry lists (k + 3 spare). Twenty near-copies of each query make the 16th upper bound
    exceed the exact 10th score: every block flags and is re-run exactly — until the first window of 32 settled blocks
    switches the handle to repair mode (r5; before it, the narrow lists switched to 32-entry ones after 64), whose
    repair pass completes these blocks in-stream: no flag after it, and the narrow lists stay. The same switch, at the
    same search, in multi-process mode (1-rank RCCL communicator: the decision comes from the exchanged flag words).
    Results are exact throughout."""
    rng = np.random.default_rng(5)
    corpus = synth.unit_norm_gaussian(91, 65536, 1024)
    q = synth.unit_norm_gaussian(92, 32, 1024)
    for i in range(32):
        near = q[i] + 1e-6 * rng.standard_normal((20, 1024)).astype(np.float32)
        corpus[1000 + 40 * i:1020 + 40 * i] = near / np.linalg.norm(near, axis=1, keepdims=True)
    ex = Index(dtype="fp32", metric="cosine")
    ex.load(corpus)
    ex.set_kernel("exact")
    want = ex.search(q, 10)
    per_mode = []
    for ix in _plain_and_dist(Index, corpus):
        flags = []
        for step in range(80):
            got = ix.search(q, 10)
            assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), step
            flags.append(ix.screen_stats()[1])
        blocks, flagged = ix.screen_stats()
        assert blocks == 80 and flagged == 32 and flags[31] == 32 and flags[30] == 31   # none after the switch
        assert ix.screen_state() == (True, 0, 0) and ix.screen_repairs() >= 48
        per_mode.append(flags)
        ix.close()
    assert per_mode[0] == per_mode[1]
    ex.close()


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_two_compute_streams_match_one(Index, devices):
    """Screened blocks alternate between two compute streams (the default): a mixed sequence of staged searches
    (several back to back, then fetched), multi-block batches, list widths that change between searches, another kind
    of search in between (k = 40), and four asynchronous searches in flight, forced re-runs included, gives, step by
    step, exactly the one-stream results."""
    corpus = synth.unit_norm_gaussian(31, 40000, 1024)
    qa = synth.unit_norm_gaussian(32, 32, 1024)
    qb = synth.unit_norm_gaussian(33, 77, 1024)
    qs = [synth.unit_norm_gaussian(34 + i, 1 + 19 * i, 1024) for i in range(6)]

    def run(streams):
        ix = Index(devices=devices, dtype="fp32", metric="cosine")
        ix.load(corpus)
        assert ix.compute_streams(streams) == streams
        out = []
        ix.set_queries(qa)
        for k in (5, 5, 7):
            ix.search_staged(k)
        out.append(ix.fetch())
        ix.set_queries(qb)
        ix.search_staged(10)
        ix.search_staged(3)
        out.append(ix.fetch())
        ix.set_queries(qa)
        for k in (5, 2, 2, 5):                     # list widths 16, 8, 8, 16
            ix.search_staged(k)
        out.append(ix.fetch())
        out.append(ix.search(qa, 40))            # large k: another kind of search between screened ones
        out.append(ix.search(qb, 12))
        tickets = [ix.search_async(q, 4 + i) for i, q in enumerate(qs[:4])]
        out += [ix.wait(t) for t in tickets]
        tickets = [ix.search_async(q, 9) for q in qs[4:]]
        ix.set_queries(qa)
        ix.search_staged(2)
        out += [ix.wait(t) for t in tickets]
        out.append(ix.fetch())
        ix.set_kernel("screen-fallback")          # every block flagged: rr_wait re-stages and re-runs exactly
        tickets = [ix.search_async(q, 6) for q in qs[:3]]
        out += [ix.wait(t) for t in tickets]
        ix.set_queries(qb)                        # flagged staged blocks, settled at the fetch: re-run exactly
        ix.search_staged(6)
        out.append(ix.fetch())
        ix.set_kernel("auto")
        tickets = []
        for q in qs:                               # the serving pattern: a new batch per search, 2 in flight
            tickets.append(ix.search_async(q, 5))
            if len(tickets) > 2:
                out.append(ix.wait(tickets.pop(0)))
        out += [ix.wait(t) for t in tickets]
        ix.close()
        return out

    for (s1, i1), (s2, i2) in zip(run(1), run(2)):
        assert np.array_equal(i1, i2) and np.array_equal(s1, s2)
