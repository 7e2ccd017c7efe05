"""Host restatement of the device merge after the candidate exchange (test infrastructure).

The device pipeline (rr_kernels.hip merge_kernel, run on every shard after the RCCL all-gather) ranks candidate
keys key = ord(score) << 32 | (0xFFFFFFFF - global_index), ord the order-preserving map of fp32 onto uint32, and
keeps the k largest: (score desc, index asc), empty slot = key 0. This restates that rule on the host so the
CPU multi-process tests check the same merge the GPU runs.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def ord_of(scores: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(scores, dtype=np.float32).view(np.uint32)
    return np.where(u & np.uint32(0x80000000), ~u, u | np.uint32(0x80000000)).astype(np.uint32)


def make_keys(scores: np.ndarray, idx: np.ndarray) -> np.ndarray:
    keys = (ord_of(scores).astype(np.uint64) << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - idx.astype(np.uint64))
    return np.where(idx >= 0, keys, np.uint64(0))


def merge_shard_topk(scores: np.ndarray, idx: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Per-shard candidates [G, b, kk] -> [b, k] by the device key order (score desc, index asc)."""
    G, b, kk = scores.shape
    keys = make_keys(scores, idx).transpose(1, 0, 2).reshape(b, G * kk)
    s = scores.transpose(1, 0, 2).reshape(b, G * kk)
    i = idx.transpose(1, 0, 2).reshape(b, G * kk)
    out_s = np.full((b, k), -np.inf, dtype=np.float32)
    out_i = np.full((b, k), -1, dtype=np.int64)
    for r in range(b):
        order = np.argsort(keys[r])[::-1]                                   # uint64 order, largest first
        order = order[keys[r][order] != 0][:k]
        out_s[r, :order.size] = s[r][order]
        out_i[r, :order.size] = i[r][order]
    return out_s, out_i
