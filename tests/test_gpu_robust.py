"""Robustness of the search pipeline's bookkeeping: the exchanged flag word, query buffers that a
re-run still needs, the ranks' agreement on the screened path, and the multi-process deadline. Every case checks
results against the one-pass exact kernel (RR_KERNEL_EXACT) of another handle on the same corpus."""
import os
import time

import numpy as np
import pytest

from oracle import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Index(hip):
    from rag_service_amd import Index as _Index
    return _Index


def _exact(Index, corpus, metric="cosine"):
    ex = Index(dtype="fp32", metric=metric)
    ex.load(corpus)
    ex.set_kernel("exact")
    return ex


def _same(got, want):
    return np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])


def test_stream_queues_distinct_and_shared_per_device(Index):
    """Hardware-queue placement (rr_stream_queues: each stream's AQL queue address, read by a probe kernel). A handle's
    four streams dispatch to four distinct hardware queues at the box's own GPU_MAX_HW_QUEUES (they take the
    high-priority pool, which nothing else of the process uses), also with a 1-rank RCCL communicator whose internal
    streams are created after them; shards on one device share one set of streams (no cross-shard stream waits).
    out[4] is the optional staging stream (rr_set_option stage_stream >= 1): none by default; made at the least
    priority (its own pool) it is distinct too."""
    import gc
    from rag_service_amd import get_unique_id
    gc.collect()                                               # handles of earlier tests released
    corpus = synth.unit_norm_gaussian(75, 4000, 512)
    one = Index(dtype="fp32", metric="cosine")
    one.load(corpus)
    qs = one.stream_queues(0)
    assert len(set(qs[:4])) == 4 and all(qs[:4]) and qs[4] == 0, [hex(v) for v in qs]
    one.set_option("stage_stream", 3)
    qs = one.stream_queues(0)
    assert len(set(qs)) == 5 and all(qs), [hex(v) for v in qs]
    one.close()
    many = Index(devices=[0, 0, 0], dtype="fp32", metric="cosine")
    many.load(corpus)
    q0 = many.stream_queues(0)
    assert len(set(q0[:4])) == 4, [hex(v) for v in q0]
    assert many.stream_queues(1) == q0 and many.stream_queues(2) == q0
    many.close()
    rx = Index(dtype="fp32", metric="cosine")
    rx.init_dist(1, 0, get_unique_id())
    rx.load(corpus)
    q = synth.unit_norm_gaussian(76, 32, 512)
    rx.search(q, 5)                                            # the communicators' streams are in use
    qr = rx.stream_queues(0)
    assert len(set(qr[:4])) == 4, [hex(v) for v in qr]
    rx.close()


def test_exchange_flag_word_cleared_between_list_widths(Index):
    """Through the RCCL exchange (1-rank communicator): k = 20 screens with 32-entry lists, so its exchanged keys
    reach past where k = 3's flag word sits (after 32 x 8 keys). Every buffer set is written at k = 20, then read
    at k = 3: without the per-block clear each k = 3 search would see a stale key as its flag and re-run exactly.
    No block may be flagged or re-run, and the results are exact."""
    from rag_service_amd import get_unique_id
    corpus = synth.unit_norm_gaussian(41, 30000, 1024)
    q = synth.unit_norm_gaussian(42, 32, 1024)
    ex = _exact(Index, corpus)
    rc = Index(dtype="fp32", metric="cosine")
    rc.init_dist(1, 0, get_unique_id())
    rc.load(corpus)
    for k in (20, 3):
        want = ex.search(q, k)
        for _ in range(6):                                    # > the 4 exchange buffer sets
            assert _same(rc.search(q, k), want), k
    blocks, flagged, reruns = rc.screen_counts()
    assert (blocks, flagged, reruns) == (12, 0, 0)
    # the one-pass path (its merge kernel writes the exchange buffer) clears the word too: exact k = 20 then k = 3
    # searches, then screened ones — a stale key merged into the result head would flag every later search
    rc.set_kernel("exact")
    for k in (20, 3):
        want = ex.search(q, k)
        for _ in range(6):
            assert _same(rc.search(q, k), want), k
    rc.set_kernel("auto")
    want = ex.search(q, 3)
    for _ in range(6):
        assert _same(rc.search(q, 3), want)
    assert rc.screen_counts() == (18, 0, 0)
    ex.close()
    rc.close()


def test_rccl_one_rank_range_guard_agreement(Index):
    """rr_init_dist handles agree on the screened path through an RCCL min at load time (finish_all): a shard with
    a value >= 2^15 turns screening off. With one rank the agreement still runs through RCCL; results exact."""
    from rag_service_amd import get_unique_id
    rng = np.random.default_rng(8)
    corpus = rng.standard_normal((5000, 512)).astype(np.float32)
    q = rng.standard_normal((32, 512)).astype(np.float32)
    ex = _exact(Index, corpus, "dot")
    rc = Index(dtype="fp32", metric="dot")
    rc.init_dist(1, 0, get_unique_id())
    rc.load(corpus)
    assert _same(rc.search(q, 5), ex.search(q, 5))
    assert rc.screen_stats() == (1, 0)
    big = corpus.copy()
    big[7, 9] = 40000.0
    rc.load(big)
    ex.load(big)
    assert _same(rc.search(q, 5), ex.search(q, 5))
    assert rc.screen_stats() == (0, 0)
    rc.close()
    ex.close()


def test_wait_rerun_keeps_the_staged_batch(Index):
    """rr_wait re-runs a flagged asynchronous search through the other query buffer and restores the staged
    batch: a batch staged with set_queries BEFORE the wait is the one the next search_staged searches."""
    corpus = synth.unit_norm_gaussian(51, 20000, 1024)
    qa = synth.unit_norm_gaussian(52, 32, 1024)
    qb = synth.unit_norm_gaussian(53, 20, 1024)
    ex = _exact(Index, corpus)
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    ix.set_kernel("screen-fallback")                           # every block flagged: rr_wait re-runs exactly
    t = ix.search_async(qb, 4)
    ix.set_queries(qa)
    assert _same(ix.wait(t), ex.search(qb, 4))
    ix.search_staged(6)
    assert _same(ix.fetch(), ex.search(qa, 6))
    assert ix.last_shape() == (32, 6)
    ix.close()
    ex.close()


def test_growing_batch_settles_the_last_search_first(Index):
    """A staged search whose block is flagged, then a LARGER batch staged (the query buffers grow and are zeroed):
    the earlier search is settled before its queries are dropped, so fetching it still gives its exact results."""
    corpus = synth.unit_norm_gaussian(61, 20000, 1024)
    qa = synth.unit_norm_gaussian(62, 32, 1024)
    qbig = synth.unit_norm_gaussian(63, 100, 1024)
    ex = _exact(Index, corpus)
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    ix.set_kernel("screen-fallback")
    ix.set_queries(qa)
    ix.search_staged(5)
    ix.set_queries(qbig)                                       # q_cap 32 -> 100: buffers reallocated
    assert _same(ix.fetch(), ex.search(qa, 5))
    ix.search_staged(5)
    assert _same(ix.fetch(), ex.search(qbig, 5))
    ix.close()
    ex.close()


@pytest.mark.parametrize("exchange", [False, True])
def test_counts_right_after_a_burst_see_every_flag(Index, exchange):
    """rr_screen_counts straight after a burst of staged searches (bench.py's window close) copies the counters and the
    last search's flag word only once every stream is idle — the flag is written by the exchange lane's merge
    (1-rank RCCL) or the last verify, on either compute stream. Every block flagged (screen-fallback): all of them are
    counted, the last search is settled (one re-run) and its results equal the exact kernel's."""
    from rag_service_amd import get_unique_id
    corpus = synth.unit_norm_gaussian(91, 125000, 1024)
    q = synth.unit_norm_gaussian(92, 32, 1024)
    ex = _exact(Index, corpus)
    ix = Index(dtype="fp32", metric="cosine")
    if exchange:
        ix.init_dist(1, 0, get_unique_id())
    ix.load(corpus)
    ix.set_queries(q)
    for _ in range(3):
        ix.search_staged(5)
    ix.synchronize()
    ix.set_kernel("screen-fallback")
    for rnd in range(3):
        b0, f0, r0, _ = ix.screen_counts_all()
        for _ in range(7):
            ix.search_staged(5)
        b1, f1, r1, _ = ix.screen_counts_all()                 # no synchronize before it
        assert (b1 - b0, f1 - f0, r1 - r0) == (7, 7, 1), (rnd, b1 - b0, f1 - f0, r1 - r0)
        assert _same(ix.fetch(), ex.search(q, 5))
    ix.close()
    ex.close()


def test_dist_deadline_fails_loudly(Index, monkeypatch):
    """The multi-process deadline (rr_set_timeout): device work that does not finish in time makes the wait return
    RR_E_TIMEOUT naming the rank, and fails the handle (later calls: RR_E_STATE). The stall is a stand-in kernel
    holding the exchange stream 1 ms per search block (option x_exchange_delay_us), after each block's all-gather, with
    a 2 ms deadline over 24 blocks; the device is left to drain before the handle is destroyed."""
    from rag_service_amd import get_unique_id
    from rag_service_amd._lib import HipRetrievalError, RR_E_STATE, RR_E_TIMEOUT
    corpus = synth.unit_norm_gaussian(71, 8000, 512)
    q = synth.unit_norm_gaussian(72, 32, 512)
    # (the exchange issue thread's short host wait for a slot's previous exchange would otherwise pace the 24 blocks
    # to the stalled lanes, leaving less than the deadline outstanding at the synchronize: x_host_wait_us = 0)
    ix = Index(dtype="fp32", metric="cosine", options={"x_exchange_delay_us": 1000, "x_host_wait_us": 0})
    ix.init_dist(1, 0, get_unique_id())
    ix.load(corpus)
    ix.search(q, 5)                                            # warm: no deadline yet (default 120 s)
    ix.set_timeout(2)
    ix.set_queries(q)
    for _ in range(24):
        ix.search_staged(5)
    t0 = time.perf_counter()
    with pytest.raises(HipRetrievalError) as e:
        ix.synchronize()
    assert e.value.code == RR_E_TIMEOUT and "rank 0 of 1" in str(e.value)
    assert time.perf_counter() - t0 < 1.0
    with pytest.raises(HipRetrievalError) as e2:
        ix.search_staged(5)
    assert e2.value.code == RR_E_STATE
    time.sleep(1.0)                                            # 24 ms of stand-in delay: the queues drain
    ix.close()
    ok = Index(dtype="fp32", metric="cosine")                  # the device is fine afterwards
    ok.load(corpus)
    ok.search(q, 5)
    ok.close()


def test_single_process_deadline_names_shard_and_stream(Index, monkeypatch):
    """Round 3's one hang (a stream that never drained, rr_search never returned) becomes a loud error: within one
    process too, every host wait polls against the handle's deadline (rr_set_timeout). Two shards on one device
    exchange by peer copies; a stand-in kernel holds the exchange lanes 1 ms per search block (x_exchange_delay_us)
    under a 2 ms deadline over 24 blocks: the wait returns RR_E_TIMEOUT naming the shard, its device and the stream,
    and the handle is failed (later calls: RR_E_STATE)."""
    from rag_service_amd._lib import HipRetrievalError, RR_E_STATE, RR_E_TIMEOUT
    corpus = synth.unit_norm_gaussian(73, 8000, 512)
    q = synth.unit_norm_gaussian(74, 32, 512)
    ix = Index(devices=[0, 0], dtype="fp32", metric="cosine", options={"x_exchange_delay_us": 1000})
    ix.load(corpus)
    ix.search(q, 5)                                            # warm, default 120 s deadline
    ix.set_timeout(2)
    ix.set_queries(q)
    for _ in range(24):
        ix.search_staged(5)
    t0 = time.perf_counter()
    with pytest.raises(HipRetrievalError) as e:
        ix.synchronize()
    msg = str(e.value)
    assert e.value.code == RR_E_TIMEOUT and "shard 0 (device 0)" in msg, msg
    assert ("compute stream" in msg or "exchange lane" in msg) and "did not complete within 2 ms" in msg, msg
    assert time.perf_counter() - t0 < 1.0
    with pytest.raises(HipRetrievalError) as e2:
        ix.search_staged(5)
    assert e2.value.code == RR_E_STATE
    time.sleep(1.0)                                            # 24 ms of stand-in delay: the queues drain
    ix.close()



@pytest.mark.parametrize("x", [False, True], ids=["local", "rccl1"])
@pytest.mark.parametrize("mode,wv", [(0, 1), (1, 0), (1, 1), (2, 1)])
def test_staging_placements_equal_the_exact_kernel(Index, mode, wv, x):
    """Where a batch is staged (option stage_stream: the next block's compute stream, or a staging stream of its own
    at normal / greatest priority) and how the compute streams follow it (stage_wait_value: an event barrier, or a
    wait-value packet on the staging's sequence word): runs of 1..8 batches staged from HBM back to back with no host
    wait in between, so each staging overlaps earlier searches; the last batch's results equal the exact kernel's.
    Also through the 1-rank RCCL exchange path."""
    torch = pytest.importorskip("torch")
    from rag_service_amd import get_unique_id
    corpus = synth.unit_norm_gaussian(91, 70000, 1024)          # >= 65536 rows: the int8 copy, its staged pieces
    qs = np.stack([synth.unit_norm_gaussian(92 + i, 32, 1024) for i in range(8)])
    dq = torch.from_numpy(qs).to("cuda:0")
    torch.cuda.synchronize()
    ex = _exact(Index, corpus)
    want = [ex.search(qs[i], 5) for i in range(8)]
    ex.close()
    ix = Index(dtype="fp32", metric="cosine", options={"stage_stream": mode, "stage_wait_value": wv})
    if x:
        ix.init_dist(1, 0, get_unique_id())
    ix.load(corpus)
    for n in range(1, 9):
        for i in range(n):
            ix.set_queries_device(dq[i].data_ptr(), 32, 1024)
            ix.search_staged(5)
        assert _same(ix.fetch(), want[n - 1]), (mode, wv, x, n)
    ix.close()
