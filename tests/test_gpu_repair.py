"""Repair mode of the screened search (rr_sk.hip "Repair"): when near-duplicate clusters defeat the
screen's lists — clusters stored contiguously fill a few workgroups' lists, so the verify cannot prove the top-k — the
handle does not re-run whole searches exactly: the screen records per chunk of rows the largest bound, the verify marks
every chunk whose bound reaches an unproven slot's exact k-th score, and an in-stream repair pass rescores exactly the
rows of those chunks and merges them with the verify's keys. The results must be BIT-IDENTICAL to the one-pass exact
kernel (RR_KERNEL_EXACT) on every case, with no host re-run."""
import numpy as np
import pytest

from test_gpu_screen import _clustered

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Index(hip):
    from rag_service_amd import Index as _Index
    return _Index


def _repair_handle(Index, monkeypatch, metric, i8, devices=None, dist=False):
    """A handle in repair mode from its load (option screen_full_lists), screening the int8 copy (i8, made for small
    corpora with screen_i8_min_rows = 0) or the f16 copy."""
    from rag_service_amd import get_unique_id
    opts = {"screen_full_lists": 1}
    if i8:
        opts["screen_i8_min_rows"] = 0
    ix = Index(devices=devices or [0], dtype="fp32", metric=metric, options=opts)
    if dist:
        ix.init_dist(1, 0, get_unique_id())
    return ix


@pytest.mark.parametrize("i8", [False, True])
@pytest.mark.parametrize("metric", ["cosine", "dot"])
@pytest.mark.parametrize("layout", ["contiguous", "interleaved"])
def test_repair_matches_exact(Index, monkeypatch, layout, metric, i8):
    """Clustered SQuAD-derived corpora (noise 0.01): repair mode returns the exact kernel's results bit for bit for
    k = 1 .. 13 (16-entry lists) and k = 20 (32-entry lists), single searches and back-to-back staged ones, and never
    flags a block; on the contiguous layout the repair pass completes query slots the lists could not prove."""
    corpus, q = _clustered(60000, 0.01, layout)
    ex = Index(dtype="fp32", metric=metric)
    ex.load(corpus)
    ex.set_kernel("exact")
    ix = _repair_handle(Index, monkeypatch, metric, i8)
    ix.load(corpus)
    assert ix.screen_state()[0] and ix.screen_int8() == i8
    for k in (1, 5, 10, 13, 20):
        want = ex.search(q, k)
        got = ix.search(q, k)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), k
        ix.set_queries(q)
        for _ in range(4):
            ix.search_staged(k)
        got = ix.fetch()
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), (k, "staged")
    blocks, flagged, reruns, wide = ix.screen_counts_all()
    repaired = ix.screen_repairs()
    print(layout, metric, i8, "blocks", blocks, "flagged", flagged, "wide", wide, "repaired", repaired)
    assert blocks == 25 and flagged == 0 and reruns == 0
    if layout == "contiguous":
        assert repaired > 0
    ix.close()
    ex.close()


@pytest.mark.parametrize("layout", ["contiguous", "interleaved"])
def test_repair_sharded_and_rccl(Index, monkeypatch, layout):
    """Repair mode through 3 shards on one device (peer-copy exchange) and through a 1-rank RCCL communicator (the
    merged keys are the shard's exchanged list): bit-identical to the exact kernel, no flagged block."""
    corpus, q = _clustered(60000, 0.01, layout)
    ex = Index(dtype="fp32", metric="cosine")
    ex.load(corpus)
    ex.set_kernel("exact")
    for devices, dist in (([0, 0, 0], False), ([0], True)):
        ix = _repair_handle(Index, monkeypatch, "cosine", True, devices=devices, dist=dist)
        ix.load(corpus)
        for k in (5, 10):
            want = ex.search(q, k)
            got = ix.search(q, k)
            assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), (devices, dist, k)
            ix.set_queries(q)
            for _ in range(3):
                ix.search_staged(k)
            got = ix.fetch()
            assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), (devices, dist, k, "staged")
        assert ix.screen_counts_all()[1] == 0
        ix.close()
    ex.close()


def test_screen_switches_to_repair_mode(Index, monkeypatch):
    """The adaptive screen: on a contiguous clustered corpus the first window of settled blocks flags (each re-run
    exactly), the handle switches to repair mode, and from then on no block flags — every result bit-identical to the
    exact kernel throughout."""
    corpus, q = _clustered(70000, 0.01, "contiguous")
    ex = Index(dtype="fp32", metric="cosine")
    ex.load(corpus)
    ex.set_kernel("exact")
    want = ex.search(q, 5)
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    assert not ix.screen_state()[0]
    flags = []
    for step in range(64):
        got = ix.search(q, 5)
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]), step
        flags.append(ix.screen_stats()[1])
    assert ix.screen_state()[0]                              # repair mode
    assert flags[-1] == flags[40] and flags[40] >= 1          # no flagged block once repairing
    assert ix.screen_repairs() > 0
    ix.close()
    ex.close()
