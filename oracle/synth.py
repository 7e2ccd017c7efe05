"""ORACLE — synthetic corpora for parity tests and benchmarks. TEST INFRASTRUCTURE ONLY.

F2 "exact-integer" corpus: x[row, col] = ((h(seed, row*d + col) mod 255) - 127) / 128
with h = splitmix64. Every value is exact in bf16 and fp32, and |dot| <= d * 127^2 / 2^14 < 2^24 / 2^14,
so every fp32 dot product is exact in any summation order: fp32, bf16 and any shard count must return
bit-identical scores. Bit-identical to the device generator (rr_fill_synthetic kind RR_SYNTH_EXACT_INT,
synth_kernel in rr_kernels.hip).

F3 "realistic" corpus: NumPy PCG64 standard normal rows, L2-normalised in fp32 — the statistics of the
reference's data/ corpora (unit-norm rows, element std ~ 1/32, SURVEY.md §2 data row).

Also: bf16 round-to-nearest-even (the corpus conversion RR_DTYPE_BF16 applies) and the device's
Irwin-Hall unit-norm generator (RR_SYNTH_UNIT_NORM), restated for host-side checks.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, i: np.ndarray) -> np.ndarray:
    """h(seed, i) = mix(seed + (i + 1) * golden), uint64 wrap-around (same as the HIP splitmix64)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i.astype(np.uint64) + np.uint64(1)) * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def exact_int_rows(seed: int, row_begin: int, n_rows: int, d: int, chunk_rows: int = 65536) -> np.ndarray:
    out = np.empty((n_rows, d), dtype=np.float32)
    for r0 in range(0, n_rows, chunk_rows):
        nr = min(chunk_rows, n_rows - r0)
        gi = (np.arange(nr * d, dtype=np.uint64) + np.uint64((row_begin + r0) * d))
        z = splitmix64(seed, gi)
        v = (z % np.uint64(255)).astype(np.int32) - 127
        out[r0:r0 + nr] = (v.astype(np.float32) * np.float32(0.0078125)).reshape(nr, d)
    return out


def exact_int_queries(seed: int, b: int, d: int) -> np.ndarray:
    """Queries from the same generator (a separate seed), exact in bf16."""
    return exact_int_rows(seed, 0, b, d)


def unit_norm_gaussian(seed: int, n: int, d: int, chunk_rows: int = 131072) -> np.ndarray:
    rng = np.random.default_rng(seed)
    out = np.empty((n, d), dtype=np.float32)
    for r0 in range(0, n, chunk_rows):
        nr = min(chunk_rows, n - r0)
        x = rng.standard_normal((nr, d), dtype=np.float32)
        x /= np.linalg.norm(x, axis=1, keepdims=True)
        out[r0:r0 + nr] = x
    return out


def irwin_hall_unnormalised(seed: int, row_begin: int, n_rows: int, d: int) -> np.ndarray:
    gi = np.arange(n_rows * d, dtype=np.uint64) + np.uint64(row_begin * d)
    z = splitmix64(seed, gi)
    m = np.uint64(0xFFFF)
    u = ((z & m).astype(np.float32) + ((z >> np.uint64(16)) & m).astype(np.float32)
         + ((z >> np.uint64(32)) & m).astype(np.float32) + (z >> np.uint64(48)).astype(np.float32))
    return ((u * np.float32(1.0 / 65536.0) - np.float32(2.0)) * np.float32(1.7320508)).reshape(n_rows, d)


def bf16_round(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 (round to nearest even) -> fp32, for finite inputs."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) << np.uint64(16)
    return r.astype(np.uint32).view(np.float32).reshape(np.shape(x))
