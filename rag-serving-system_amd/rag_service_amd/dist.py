"""One-process-per-GPU coordination for a row-sharded corpus.

The data path (candidate exchange) is RCCL inside librag_retrieval.so (ncclAllGather over xGMI). This
module is only the control plane around it: rank/world from the torchrun environment, broadcasting the
RCCL unique id, and reductions of host-side timings. It uses a CPU `gloo` process group so it never
creates a second GPU communicator.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional, Tuple


def env_rank_world() -> Tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard_rows(n: int, world: int, g: int) -> Tuple[int, int]:
    """Rows [begin, end) of global shard g (same formula as rr_api.cpp shard_range)."""
    per = (n + world - 1) // world
    b = min(n, g * per)
    return b, min(n, b + per)


def init_control_plane(world: int, rank: int, timeout_s: int = 300):
    """gloo process group from MASTER_ADDR/PORT (torchrun env); None when world == 1."""
    if world <= 1:
        return None
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    return dist


def broadcast_bytes(dist, payload: Optional[bytes], src: int = 0) -> bytes:
    obj = [payload]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


def all_gather_bytes(dist, payload: Optional[bytes]) -> list:
    """Every rank's payload, in rank order (world == 1: [payload])."""
    if dist is None:
        return [payload]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, payload)
    return out


def placement(n_docs: int, world: int, shard_group: int = 0, min_shard_rows: int = 500_000) -> Tuple[int, int]:
    """(S, R): the ranks are split into R replica groups of S consecutive ranks; each group holds the whole corpus as S
    contiguous row shards (one RCCL communicator per group: the per-block all-gather of candidates and the device
    merge) and searches its own batches. shard_group > 0 fixes S; 0 (auto) takes the fewest ranks whose
    shards still have >= min_shard_rows rows each — below that a shard's per-block fixed cost (screen start-up and
    tail, the verify and staging chain: DESIGN §5 "Placement") outweighs the bytes it streams — and S is rounded up
    to a divisor of world."""
    if world <= 1:
        return 1, 1
    s = shard_group if shard_group > 0 else max(1, -(-n_docs // max(1, min_shard_rows)))
    s = min(max(1, s), world)
    while world % s:
        s += 1
    return s, world // s


def max_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier(dist) -> None:
    if dist is not None:
        dist.barrier()
