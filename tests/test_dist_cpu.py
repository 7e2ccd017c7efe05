"""Multi-process control plane on CPU (gloo, world_size 2): the pieces of the N>1 path that do not need a
GPU — shard partition, RCCL unique-id broadcast, max-over-ranks timing, and the merge rule that makes
sharded results identical to the single-shard result (tests/dist_helpers.py restates the device merge's key
order; checked against the oracle)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle.retriever_oracle import canonical_topk, exact_scores
from dist_helpers import merge_shard_topk
from rag_service_amd.dist import shard_rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from rag_service_amd.dist import (barrier, broadcast_bytes, env_rank_world, init_control_plane,
                                      max_over_ranks)
    r, w, local = env_rank_world()
    dist = init_control_plane(w, r)
    uid = broadcast_bytes(dist, bytes(range(128)) if r == 0 else None)
    t = max_over_ranks(dist, float(r + 1) * 0.5)
    barrier(dist)
    # each rank scores its shard with the oracle and the shards are merged on every rank
    rng = np.random.default_rng(3)
    corpus = rng.standard_normal((1000, 64)).astype(np.float32)
    queries = rng.standard_normal((5, 64)).astype(np.float32)
    b0, b1 = shard_rows(corpus.shape[0], w, r)
    sv, si = canonical_topk(exact_scores(corpus[b0:b1], queries, "dot"), 7)
    si = np.where(si >= 0, si + b0, -1)
    import torch
    gathered = [None] * w
    dist.all_gather_object(gathered, (sv.astype(np.float32), si))
    ms, mi = merge_shard_topk(np.stack([g[0] for g in gathered]), np.stack([g[1] for g in gathered]), 7)
    q.put((r, uid, t, mi))
    dist.destroy_process_group()


def test_gloo_world2_control_plane_and_merge():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(3)
    corpus = rng.standard_normal((1000, 64)).astype(np.float32)
    queries = rng.standard_normal((5, 64)).astype(np.float32)
    _, want = canonical_topk(exact_scores(corpus, queries, "dot"), 7)
    for r, uid, t, mi in out:
        assert uid == bytes(range(128))
        assert t == 1.0
        assert np.array_equal(mi, want)


@pytest.mark.parametrize("n,world", [(1_000_000, 8), (10, 8), (7, 3), (33, 2), (1, 4)])
def test_shard_rows_partition(n, world):
    spans = [shard_rows(n, world, g) for g in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0 and a0 <= a1
    assert sum(e - b for b, e in spans) == n


def test_host_merge_equals_single_shard():
    rng = np.random.default_rng(11)
    corpus = rng.standard_normal((2000, 32)).astype(np.float32)
    q = rng.standard_normal((4, 32)).astype(np.float32)
    ex = exact_scores(corpus, q, "cosine")
    want_v, want_i = canonical_topk(ex, 12)
    for world in (2, 3, 8):
        vs, ids = [], []
        for g in range(world):
            b0, b1 = shard_rows(corpus.shape[0], world, g)
            v, i = canonical_topk(ex[:, b0:b1], 12)
            vs.append(v.astype(np.float32))
            ids.append(np.where(i >= 0, i + b0, -1))
        mv, mi = merge_shard_topk(np.stack(vs), np.stack(ids), 12)
        assert np.array_equal(mi, want_i)


class _FakeIndex:
    """Stands in for rag_service_amd.Index in bench.timed_steps (no GPU): every screened search block flags with the
    rank's own rate, the library re-runs some of them itself, and each search issued under kernel "exact" is counted
    (the re-runs timed_steps pays)."""

    def __init__(self, flag_every, lib_rerun_every):
        self.kernel = "auto"
        self.blocks = self.flagged = self.reruns = 0
        self.exact_searches = 0
        self.flag_every, self.lib_rerun_every = flag_every, lib_rerun_every

    def search_staged(self, k):
        if self.kernel == "exact":
            self.exact_searches += 1
            return
        self.blocks += 1
        if self.flag_every and self.blocks % self.flag_every == 0:
            self.flagged += 1
            if self.lib_rerun_every and self.flagged % self.lib_rerun_every == 0:
                self.reruns += 1

    def synchronize(self):
        pass

    def screen_counts_all(self):
        return self.blocks, self.flagged, self.reruns, 0

    def set_timing(self, on):
        pass

    def kernel_time(self, reset=True):
        return 0.0, 0

    def set_kernel(self, k):
        self.kernel = k


def _timed_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from rag_service_amd.dist import init_control_plane
    dist = init_control_plane(world, rank)
    # rank 0: every 4th block flags, the library re-runs every 2nd flagged one; rank 1: every 5th, none re-run
    ix = _FakeIndex(4, 2) if rank == 0 else _FakeIndex(5, 0)
    acct = {}
    bench.timed_steps(ix, 5, 40, 3, dist, lambda: None, 1, acct)
    q.put((rank, acct, ix.exact_searches))
    dist.destroy_process_group()


def test_timed_steps_pays_summed_reruns_on_every_rank():
    """bench.timed_steps at world 2 (gloo, a fake index per rank): the blocks each rank flagged inside the window and
    the library did not re-run itself are summed over the ranks, and EVERY rank issues that many exact searches
    before the closing sync — so their all-gathers pair up. Rank 0: 40 window blocks, 10 flagged (every
    4th), 5 re-run by the library -> owes 5; rank 1: 8 flagged, none re-run -> owes 8; both pay 13."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_timed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, a0, e0), (r1, a1, e1) = out
    assert (a0["blocks"], a0["flagged"], a0["reruns_library"]) == (40, 10, 5)
    assert (a1["blocks"], a1["flagged"], a1["reruns_library"]) == (40, 8, 0)
    assert a0["reruns_paid"] == a1["reruns_paid"] == 13 and e0 == e1 == 13
