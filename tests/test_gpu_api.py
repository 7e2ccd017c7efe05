"""C-ABI behaviour beyond the kernels: the RCCL exchange with a 1-rank communicator, reloads, result shapes,
the pipelined async search."""
import numpy as np
import pytest

from oracle.retriever_oracle import canonical_topk, exact_scores
from parity_helpers import check_topk

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib(hip):
    import rag_service_amd
    return rag_service_amd


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_rccl_one_rank_exchange_matches_single_shard(lib, dtype):
    """rr_init_dist(world=1) creates a real RCCL communicator, so every search takes the all-gather exchange:
    the pipelined branch (k <= 32, exchange stream, parity buffers) and the serial one (k > 32). Results must be
    bit-identical to the handle without an exchange, over back-to-back staged searches and mixed k."""
    rng = np.random.default_rng(3)
    corpus = rng.standard_normal((7001, 1024)).astype(np.float32)
    q = rng.standard_normal((45, 1024)).astype(np.float32)     # two query blocks
    plain = lib.Index(devices=[0], dtype=dtype, metric="cosine")
    plain.load(corpus)
    rc = lib.Index(devices=[0], dtype=dtype, metric="cosine")
    rc.init_dist(1, 0, lib.get_unique_id())
    assert rc.dist_info() == (1, 0)
    assert plain.dist_info() == (0, -1)
    rc.load(corpus)
    for k in (5, 40, 8, 32, 33, 1):
        want = plain.search(q, k)
        got = rc.search(q, k)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), k
    rc.set_queries(q)
    for k in (5, 40, 5, 5):
        for _ in range(3):
            rc.search_staged(k)
        s, i = rc.fetch()
        want = plain.search(q, k)
        assert np.array_equal(i, want[1]) and np.array_equal(s, want[0]), k
    plain.close()
    rc.close()


def test_reload_with_other_dim_and_size(lib):
    """A handle reloaded with a different d / row count drops its work buffers (they were sized for the old
    corpus): searches after the reload are correct, and the staged batch does not survive the reload."""
    rng = np.random.default_rng(4)
    ix = lib.Index(dtype="fp32", metric="cosine")
    c1 = rng.standard_normal((300, 64)).astype(np.float32)
    q1 = rng.standard_normal((70, 64)).astype(np.float32)
    ix.load(c1)
    ix.search(q1, 5)
    c2 = rng.standard_normal((5000, 1024)).astype(np.float32)
    q2 = rng.standard_normal((40, 1024)).astype(np.float32)
    ix.load(c2)
    with pytest.raises(lib.HipRetrievalError):
        ix.search_staged(5)                         # the 64-d batch staged before the reload is gone
    s, i = ix.search(q2, 7)
    _, cidx = canonical_topk(exact_scores(c2, q2, "cosine"), 7)
    check_topk(i, s, cidx, c2, q2, "cosine", near_tie=1e-5 * 32, score_tol=1e-3)
    ix.load(c1)                                     # and back to the small one
    s, i = ix.search(q1, 3)
    _, cidx = canonical_topk(exact_scores(c1, q1, "cosine"), 3)
    check_topk(i, s, cidx, c1, q1, "cosine", near_tie=1e-5 * 8, score_tol=1e-3)
    ix.close()


def test_fetch_returns_the_last_search_shape(lib):
    rng = np.random.default_rng(5)
    corpus = rng.standard_normal((2000, 256)).astype(np.float32)
    ix = lib.Index(dtype="fp32", metric="dot")
    ix.load(corpus)
    ix.set_queries(corpus[:1])
    ix.search_staged(1)
    assert ix.last_shape() == (1, 1)
    q = rng.standard_normal((64, 256)).astype(np.float32)
    s, i = ix.search(q, 100)                        # synchronous search after a staged one
    assert ix.last_shape() == (64, 100)
    s2, i2 = ix.fetch()
    assert s2.shape == (64, 100) and np.array_equal(i2, i) and np.array_equal(s2, s)
    ix.close()


@pytest.mark.parametrize("shards", [1, 3])
def test_async_pipeline_matches_sync(lib, shards):
    rng = np.random.default_rng(6)
    corpus = rng.standard_normal((9000, 512)).astype(np.float32)
    ix = lib.Index(devices=[0] * shards, dtype="fp32", metric="cosine")
    ix.load(corpus)
    batches = [(rng.standard_normal((b, 512)).astype(np.float32), k)
               for b, k in [(32, 5), (7, 40), (64, 10), (1, 1), (33, 32), (32, 5)]]
    want = [ix.search(q, k) for q, k in batches]
    tickets = [ix.search_async(q, k) for q, k in batches[:4]]
    with pytest.raises(lib.HipRetrievalError):
        ix.search_async(*batches[4])                # four already in flight
    got = [ix.wait(t) for t in tickets[:2]]
    tickets += [ix.search_async(q, k) for q, k in batches[4:]]
    got += [ix.wait(t) for t in tickets[2:]]
    for (ws, wi), (gs, gi) in zip(want, got):
        assert np.array_equal(wi, gi) and np.array_equal(ws, gs)
    with pytest.raises(lib.HipRetrievalError):     # a ticket is waited exactly once
        lib._lib._check(ix._lib.rr_wait(ix._h, tickets[0], gs.ctypes.data_as(lib._lib._fp),
                                        gi.ctypes.data_as(lib._lib._i64p)))
    ix.close()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp32-split"])
def test_update_rows_equals_reload(lib, dtype, devices):
    """rr_update_rows overwrites rows in place — storage conversion, per-row norms, the screening copy — so a handle
    updated in place answers bit-identically to one loaded with the modified corpus, for both metrics and every k
    path (screened k <= 29 for fp32, k > 32), across shard boundaries and with a repeated index (the last row wins).
    A row beyond the f16 range turns the screened search off (the exact kernel's results, still identical)."""
    rng = np.random.default_rng(11)
    n, d = 6007, 512
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((40, d)).astype(np.float32)
    idx = np.array([0, 17, 2002, 2003, 4005, n - 1, 17], dtype=np.int64)
    new = rng.standard_normal((len(idx), d)).astype(np.float32)
    new[1] = q[3] * 2.0                              # overwritten again by the repeated index below
    new[-1] = q[5] * 0.5                             # row 17 becomes a near-copy of query 5
    changed = corpus.copy()
    for r, row in zip(idx, new):
        changed[r] = row
    for metric in ("cosine", "dot"):
        up = lib.Index(devices=devices, dtype=dtype, metric=metric)
        up.load(corpus)
        up.search(q, 5)
        up.update_rows(new, idx)
        fresh = lib.Index(devices=devices, dtype=dtype, metric=metric)
        fresh.load(changed)
        for k in (5, 12, 40):
            want = fresh.search(q, k)
            got = up.search(q, k)
            assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), (metric, k)
        assert up.read_rows(17, 1).tobytes() == fresh.read_rows(17, 1).tobytes()
        if dtype == "fp32":                          # |x| >= 2^15: the screen's f16 reading cannot hold it
            big = np.zeros((1, d), np.float32)
            big[0, 0] = 40000.0
            up.update_rows(big, np.array([9], np.int64))
            changed2 = changed.copy()
            changed2[9] = big[0]
            ex = lib.Index(devices=devices, dtype=dtype, metric=metric)
            ex.load(changed2)
            ex.set_kernel("exact")
            want = ex.search(q, 5)
            blocks0 = up.screen_stats()[0]
            got = up.search(q, 5)
            assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), metric
            assert up.screen_stats()[0] == blocks0   # no screened block ran
            ex.close()
        up.close()
        fresh.close()


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_update_rows_refreshes_the_int8_copy(lib, monkeypatch, devices):
    """rr_update_rows on a handle that screens the int8 copy (RR_SCREEN_I8_MIN_ROWS=0: the copy is made for this small
    corpus; d = 1024): the updated rows' int8 values, scales and error norms (store_rows -> f32_to_i8_kernel on single
    rows) are refreshed in place, so the int8 screen's bound stays valid for them — results bit-identical to a handle
    loaded with the modified corpus and to the exact kernel, rows that became the queries' best matches included
    (a stale int8 row would drop true top-k rows without any flag)."""
    rng = np.random.default_rng(12)
    n, d = 5003, 1024
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((32, d)).astype(np.float32)
    idx = np.array([3, 1999, 2501, 2502, n - 1, 4000], dtype=np.int64)
    new = rng.standard_normal((len(idx), d)).astype(np.float32)
    for j, r in enumerate(idx[:4]):                  # near-copies of queries: each becomes its query's top row
        new[j] = q[2 * j] + 0.01 * rng.standard_normal(d).astype(np.float32)
    new[5, 7] = 25.0                                 # a spike: every other element of its int8 row rounds to 0
    changed = corpus.copy()
    changed[idx] = new
    for metric in ("cosine", "dot"):
        monkeypatch.setenv("RR_SCREEN_I8_MIN_ROWS", "0")
        up = lib.Index(devices=devices, dtype="fp32", metric=metric)
        fresh = lib.Index(devices=devices, dtype="fp32", metric=metric)
        monkeypatch.delenv("RR_SCREEN_I8_MIN_ROWS")
        up.load(corpus)
        up.search(q, 5)
        up.update_rows(new, idx)
        fresh.load(changed)
        assert up.screen_int8() and fresh.screen_int8()
        ex = lib.Index(devices=devices, dtype="fp32", metric=metric)
        ex.load(changed)
        ex.set_kernel("exact")
        for k in (1, 5, 10):
            want = ex.search(q, k)
            for h in (up, fresh):
                got = h.search(q, k)
                assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), (metric, k)
        assert all(want[1][2 * j, 0] == idx[j] for j in range(4)) or metric == "dot"
        assert up.screen_int8()                      # still screening the int8 copy
        for h in (up, fresh, ex):
            h.close()


def test_wait_settles_its_search_once(lib, monkeypatch):
    """rr_wait settles the search of its ticket: a later rr_synchronize / rr_fetch_results does not observe it a
    second time (the adaptive screen's windows count it once) nor re-run a flagged one again. Forced
    fallbacks (RR_KERNEL_SCREEN_FALLBACK) flag every block: one wait = one re-run, then a synchronize adds none."""
    rng = np.random.default_rng(13)
    corpus = rng.standard_normal((4099, 512)).astype(np.float32)
    q = rng.standard_normal((32, 512)).astype(np.float32)
    ix = lib.Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    want = ix.search(q, 5)
    ix.set_kernel("screen-fallback")
    _, f0, r0, _ = ix.screen_counts_all()
    got = ix.wait(ix.search_async(q, 5))
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    ix.synchronize()
    _, f1, r1, _ = ix.screen_counts_all()
    assert (f1 - f0, r1 - r0) == (1, 1)
    ix.close()
