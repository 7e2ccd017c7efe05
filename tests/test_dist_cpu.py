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
