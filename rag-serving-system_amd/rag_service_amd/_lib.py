"""ctypes binding of the C-ABI in include/rag_retrieval.h (librag_retrieval.so, built in-tree).

No PyTorch and no CPU fallback: if the shared library is missing or fails to load, every entry point
raises ``HipRetrievalUnavailable``. The product path never routes through ``oracle/``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
import threading
from typing import Optional, Sequence, Tuple

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # rag-serving-system_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
# RR_LIBRARY: another build of the same library (A/B measurements of kernel variants in one box call)
LIB_PATH = os.environ.get("RR_LIBRARY") or os.path.join(PKG_ROOT, "librag_retrieval.so")
HEADER_PATH = os.path.join(REPO_ROOT, "include", "rag_retrieval.h")

# mirrors include/rag_retrieval.h
RR_OK = 0
RR_E_INVALID = -1
RR_E_HIP = -2
RR_E_RCCL = -3
RR_E_STATE = -4
RR_E_UNSUPPORTED = -5
RR_E_OOM = -6
RR_E_TIMEOUT = -7
RR_DTYPE_F32 = 0
RR_DTYPE_BF16 = 1
RR_DTYPE_F32_SPLIT = 2
RR_METRIC_DOT = 0
RR_METRIC_COSINE = 1
RR_SYNTH_EXACT_INT = 0
RR_SYNTH_UNIT_NORM = 1
RR_UNIQUE_ID_BYTES = 128
RR_FUSED_KMAX = 32
RR_KERNEL_AUTO = 0
RR_KERNEL_FUSED = 1
RR_KERNEL_EXACT = 2
RR_KERNEL_SCREEN_FALLBACK = 3
RR_ABI_VERSION = 9

DTYPES = {"fp32": RR_DTYPE_F32, "float32": RR_DTYPE_F32, "f32": RR_DTYPE_F32,
          "bf16": RR_DTYPE_BF16, "bfloat16": RR_DTYPE_BF16, "fp32-split": RR_DTYPE_F32_SPLIT}
METRICS = {"dot": RR_METRIC_DOT, "cosine": RR_METRIC_COSINE}

# Every function the header declares: name -> (restype, argtypes)
_c_int, _c_i32, _c_i64, _c_u64 = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
_vp, _fp, _i64p, _ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)
SIGNATURES = {
    "rr_create": (_c_int, [_ip, _c_int, _c_int, _c_int, ctypes.POINTER(_vp)]),
    "rr_destroy": (None, [_vp]),
    "rr_last_error": (ctypes.c_char_p, []),
    "rr_abi_version": (_c_int, []),
    "rr_get_unique_id": (_c_int, [ctypes.c_char_p]),
    "rr_init_dist": (_c_int, [_vp, _c_int, _c_int, ctypes.c_char_p]),
    "rr_load": (_c_int, [_vp, _fp, _c_i64, _c_i32]),
    "rr_load_rows": (_c_int, [_vp, _fp, _c_i64, _c_i64, _c_i64, _c_i32]),
    "rr_fill_synthetic": (_c_int, [_vp, _c_int, _c_u64, _c_i64, _c_i32]),
    "rr_info": (_c_int, [_vp, _i64p, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32)]),
    "rr_shard_range": (_c_int, [_vp, _c_int, _i64p, _i64p]),
    "rr_read_rows": (_c_int, [_vp, _c_i64, _c_i64, _fp]),
    "rr_search": (_c_int, [_vp, _fp, _c_i32, _c_i32, _c_i32, _fp, _i64p]),
    "rr_set_queries": (_c_int, [_vp, _fp, _c_i32, _c_i32]),
    "rr_search_staged": (_c_int, [_vp, _c_i32]),
    "rr_synchronize": (_c_int, [_vp]),
    "rr_fetch_results": (_c_int, [_vp, _fp, _i64p]),
    "rr_set_queries_device": (_c_int, [_vp, _vp, _c_i32, _c_i32]),
    "rr_set_kernel": (_c_int, [_vp, _c_int]),
    "rr_set_timing": (_c_int, [_vp, _c_int]),
    "rr_kernel_time": (_c_int, [_vp, ctypes.POINTER(ctypes.c_double), _i64p, _c_int]),
    "rr_search_async": (_c_int, [_vp, _fp, _c_i32, _c_i32, _c_i32, ctypes.POINTER(_c_i32)]),
    "rr_wait": (_c_int, [_vp, _c_i32, _fp, _i64p]),
    "rr_screen_stats": (_c_int, [_vp, _i64p, _i64p]),
    "rr_set_schedule": (_c_int, [_vp, _c_int]),
    "rr_screen_copy": (_c_int, [_vp, _c_i32, ctypes.POINTER(_c_i32)]),
    "rr_screen_int8": (_c_int, [_vp, _c_i32, ctypes.POINTER(_c_i32)]),
    "rr_set_compute_streams": (_c_int, [_vp, _c_i32, ctypes.POINTER(_c_i32)]),
    "rr_last_shape": (_c_int, [_vp, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32)]),
    "rr_dist_info": (_c_int, [_vp, _ip, _ip]),
    "rr_screen_counts": (_c_int, [_vp, _i64p, _i64p, _i64p, _i64p]),
    "rr_set_timeout": (_c_int, [_vp, _c_i32]),
    "rr_stream_queues": (_c_int, [_vp, _c_int, ctypes.POINTER(ctypes.c_uint64)]),
    "rr_update_rows": (_c_int, [_vp, _fp, _i64p, _c_i64, _c_i32]),
    "rr_screen_state": (_c_int, [_vp, ctypes.POINTER(_c_i32), _i64p, _i64p]),
    "rr_screen_repairs": (_c_int, [_vp, _i64p]),
    "rr_screen_factors": (_c_int, [_vp, _c_i64, _c_i64, _fp, _fp, _fp]),
    "rr_set_option": (_c_int, [_vp, ctypes.c_char_p, _c_i64]),
    "rr_get_option": (_c_int, [_vp, ctypes.c_char_p, _i64p]),
    "rr_build_info": (ctypes.c_char_p, []),
}


class HipRetrievalUnavailable(RuntimeError):
    """The HIP extension is not built or cannot be loaded (there is no CPU fallback)."""


class HipRetrievalError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rr error {code}: {msg}")
        self.code = code


_lib = None
_lib_lock = threading.Lock()


def build(force: bool = False) -> str:
    """Compile librag_retrieval.so for gfx950 with hipcc (in-tree)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-C", PKG_ROOT, "-j8"])
    return LIB_PATH


def load_library(path: Optional[str] = None):
    """Load (once) and type the shared library. Raises HipRetrievalUnavailable if absent."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        # If the caller already imported torch (its wheel bundles its own libamdhip64.so.7), let torch
        # bring up the HIP runtime first so both share one runtime instance in this process.
        torch = sys.modules.get("torch")
        if torch is not None:
            try:
                torch.cuda.is_available()
            except Exception:
                pass
        if not os.path.exists(p):
            raise HipRetrievalUnavailable(
                f"{p} not found: build it with `make -C {PKG_ROOT}` (hipcc --offload-arch=gfx950)")
        try:
            lib = ctypes.CDLL(p)
        except OSError as e:
            raise HipRetrievalUnavailable(f"cannot load {p}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.rr_abi_version() != RR_ABI_VERSION:
            raise HipRetrievalUnavailable("ABI version mismatch")
        if path is None:
            _lib = lib
        return lib


def _check(rc: int) -> None:
    if rc != RR_OK:
        msg = load_library().rr_last_error().decode(errors="replace")
        raise HipRetrievalError(rc, msg)


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(_fp)


def _i64ptr(a: np.ndarray):
    return a.ctypes.data_as(_i64p)


def build_info() -> str:
    """The library's build: "gfx950; product build", or an A/B build's description (RR_AB_ENV)."""
    return load_library().rr_build_info().decode()


def get_unique_id() -> bytes:
    lib = load_library()
    buf = ctypes.create_string_buffer(RR_UNIQUE_ID_BYTES)
    _check(lib.rr_get_unique_id(buf))
    return buf.raw


class Index:
    """Owning wrapper of one ``rr_handle``: a (possibly sharded) corpus resident in HBM.

    The arithmetic contract is the C-ABI's: results sorted by (score desc, index asc); slots beyond
    the corpus size hold (-inf, -1).
    """

    def __init__(self, devices: Optional[Sequence[int]] = None, dtype: str = "fp32", metric: str = "cosine",
                 options: Optional[dict] = None):
        """options: path settings applied right after creation (rr_set_option; results are the same under any)."""
        self._lib = load_library()
        if dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {sorted(DTYPES)}")
        if metric not in METRICS:
            raise ValueError(f"metric must be one of {sorted(METRICS)}")
        self.dtype, self.metric = dtype, metric
        h = _vp()
        if devices is None:
            _check(self._lib.rr_create(None, 1, DTYPES[dtype], METRICS[metric], ctypes.byref(h)))
        else:
            arr = (ctypes.c_int * len(devices))(*devices)
            _check(self._lib.rr_create(arr, len(devices), DTYPES[dtype], METRICS[metric], ctypes.byref(h)))
        self._h = h
        self.n = 0
        self.d = 0
        self.kernel = "auto"
        self._tickets = {}
        for name, value in (options or {}).items():
            self.set_option(name, value)

    # -- lifecycle ---------------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.rr_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def init_dist(self, world: int, rank: int, unique_id: bytes) -> None:
        _check(self._lib.rr_init_dist(self._h, world, rank, unique_id))

    def dist_info(self) -> Tuple[int, int]:
        """(ranks in the RCCL communicator, this process's rank): (0, -1) without one."""
        n, r = ctypes.c_int(), ctypes.c_int()
        _check(self._lib.rr_dist_info(self._h, ctypes.byref(n), ctypes.byref(r)))
        return n.value, r.value

    # -- corpus ------------------------------------------------------------------------------------
    def load(self, corpus: np.ndarray) -> None:
        c = np.ascontiguousarray(corpus, dtype=np.float32)
        if c.ndim != 2:
            raise ValueError("corpus must be 2-D")
        _check(self._lib.rr_load(self._h, _fptr(c), c.shape[0], c.shape[1]))
        self.n, self.d = c.shape

    def load_rows(self, rows: np.ndarray, row_begin: int, n_total: int) -> None:
        r = np.ascontiguousarray(rows, dtype=np.float32)
        _check(self._lib.rr_load_rows(self._h, _fptr(r), row_begin, r.shape[0], n_total, r.shape[1]))
        self.n, self.d = n_total, r.shape[1]

    def fill_synthetic(self, kind: int, seed: int, n: int, d: int) -> None:
        _check(self._lib.rr_fill_synthetic(self._h, kind, seed, n, d))
        self.n, self.d = n, d

    def info(self) -> Tuple[int, int, int, int]:
        n, d, nl, w = _c_i64(), _c_i32(), _c_i32(), _c_i32()
        _check(self._lib.rr_info(self._h, ctypes.byref(n), ctypes.byref(d), ctypes.byref(nl), ctypes.byref(w)))
        return n.value, d.value, nl.value, w.value

    def shard_range(self, i: int = 0) -> Tuple[int, int]:
        b, e = _c_i64(), _c_i64()
        _check(self._lib.rr_shard_range(self._h, i, ctypes.byref(b), ctypes.byref(e)))
        return b.value, e.value

    def update_rows(self, rows: np.ndarray, row_idx) -> None:
        """Overwrite the corpus rows at the given global indices in place (rr_update_rows)."""
        r = np.ascontiguousarray(rows, dtype=np.float32)
        ix = np.ascontiguousarray(row_idx, dtype=np.int64)
        if r.ndim != 2 or ix.ndim != 1 or r.shape[0] != ix.shape[0]:
            raise ValueError("rows must be (n, d) with one index per row")
        _check(self._lib.rr_update_rows(self._h, _fptr(r), _i64ptr(ix), r.shape[0], r.shape[1]))

    def read_rows(self, row_begin: int, n_rows: int) -> np.ndarray:
        out = np.empty((n_rows, self.d), dtype=np.float32)
        _check(self._lib.rr_read_rows(self._h, row_begin, n_rows, _fptr(out)))
        return out

    # -- search ------------------------------------------------------------------------------------
    def search(self, queries: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim != 2:
            raise ValueError("queries must be 2-D")
        b = q.shape[0]
        scores = np.empty((b, k), dtype=np.float32)
        idx = np.empty((b, k), dtype=np.int64)
        _check(self._lib.rr_search(self._h, _fptr(q), b, q.shape[1], k, _fptr(scores), _i64ptr(idx)))
        return scores, idx

    def search_async(self, queries: np.ndarray, k: int) -> int:
        """Enqueue H2D + search + D2H of one batch; returns a ticket for wait() (at most 4 in flight)."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim != 2:
            raise ValueError("queries must be 2-D")
        t = _c_i32()
        _check(self._lib.rr_search_async(self._h, _fptr(q), q.shape[0], q.shape[1], k, ctypes.byref(t)))
        self._tickets[t.value] = (q.shape[0], k)
        return t.value

    def wait(self, ticket: int) -> Tuple[np.ndarray, np.ndarray]:
        b, k = self._tickets.pop(ticket)
        scores = np.empty((b, k), dtype=np.float32)
        idx = np.empty((b, k), dtype=np.int64)
        _check(self._lib.rr_wait(self._h, ticket, _fptr(scores), _i64ptr(idx)))
        return scores, idx

    def set_queries(self, queries: np.ndarray) -> None:
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim != 2:
            raise ValueError("queries must be 2-D")
        _check(self._lib.rr_set_queries(self._h, _fptr(q), q.shape[0], q.shape[1]))

    def set_queries_device(self, dev_ptr: int, b: int, d: int) -> None:
        _check(self._lib.rr_set_queries_device(self._h, _vp(dev_ptr), b, d))

    def search_staged(self, k: int) -> None:
        _check(self._lib.rr_search_staged(self._h, k))

    def synchronize(self) -> None:
        _check(self._lib.rr_synchronize(self._h))

    def last_shape(self) -> Tuple[int, int]:
        """(batch, k) of the last search: the shape fetch() returns."""
        b, k = _c_i32(), _c_i32()
        _check(self._lib.rr_last_shape(self._h, ctypes.byref(b), ctypes.byref(k)))
        return b.value, k.value

    def fetch(self) -> Tuple[np.ndarray, np.ndarray]:
        """Results of the LAST search (staged or synchronous), sized from the C side's own record."""
        b, k = self.last_shape()
        if b < 1 or k < 1:
            raise HipRetrievalError(RR_E_STATE, "no search has run")
        scores = np.empty((b, k), dtype=np.float32)
        idx = np.empty((b, k), dtype=np.int64)
        _check(self._lib.rr_fetch_results(self._h, _fptr(scores), _i64ptr(idx)))
        return scores, idx

    KERNELS = {"auto": RR_KERNEL_AUTO, "fused": RR_KERNEL_FUSED, "exact": RR_KERNEL_EXACT,
               "screen-fallback": RR_KERNEL_SCREEN_FALLBACK}

    def set_kernel(self, kernel: str) -> None:
        """'auto' (split-K LDS-DMA kernel where the shape allows; the screened search for fp32 storage and 64-slot bf16 blocks),
        'exact' (split-K, fp32 scored exactly in one pass), 'fused' (register-streaming kernel) or
        'screen-fallback' (test hook: the screened search's exact fallback pass always runs)."""
        _check(self._lib.rr_set_kernel(self._h, self.KERNELS[kernel]))
        self.kernel = kernel

    def set_schedule(self, dynamic: bool) -> None:
        """Split-K work schedule: dynamic chunk counter (default) or static round-robin chunks."""
        _check(self._lib.rr_set_schedule(self._h, 1 if dynamic else 0))

    def compute_streams(self, n: Optional[int] = None) -> int:
        """Screened search blocks on 2 alternating compute streams (the default) or 1 (results identical); None
        leaves the setting. Returns the streams in use."""
        u = _c_i32()
        _check(self._lib.rr_set_compute_streams(self._h, -1 if n is None else int(n), ctypes.byref(u)))
        return u.value

    def screen_copy(self, use: Optional[bool] = None) -> bool:
        """The screened search's f16 copy of fp32 rows (half the bytes per screen pass; results unchanged):
        use=True keeps one from the next load, False frees it; returns whether it is in use."""
        p = _c_i32()
        _check(self._lib.rr_screen_copy(self._h, -1 if use is None else int(bool(use)), ctypes.byref(p)))
        return bool(p.value)

    def screen_int8(self, use: Optional[bool] = None) -> bool:
        """The screened search's int8 copy (a quarter of the fp32 bytes per screen pass, a looser bound; results
        unchanged): use=True screens it (re-armed), False screens the f16 copy; returns whether the next search
        screens the int8 copy."""
        p = _c_i32()
        _check(self._lib.rr_screen_int8(self._h, -1 if use is None else int(bool(use)), ctypes.byref(p)))
        return bool(p.value)

    def screen_repairs(self) -> int:
        """Query slots the repair pass completed (repair mode) since the corpus was loaded, over local shards."""
        n = _c_i64()
        _check(self._lib.rr_screen_repairs(self._h, ctypes.byref(n)))
        return n.value

    def screen_stats(self) -> Tuple[int, int]:
        """(screened search blocks, blocks that needed the exact fallback pass)."""
        b, f = _c_i64(), _c_i64()
        _check(self._lib.rr_screen_stats(self._h, ctypes.byref(b), ctypes.byref(f)))
        return b.value, f.value

    def screen_counts(self) -> Tuple[int, int, int]:
        """(screened search blocks, blocks flagged for the exact pass, exact re-runs the handle ran). Flagged
        blocks of staged searches that were superseded before anyone fetched them are never re-run; a benchmark
        pays flagged - re-runs exact searches itself."""
        return self.screen_counts_all()[:3]

    def screen_counts_all(self) -> Tuple[int, int, int, int]:
        """screen_counts() plus the query slots the verify proved only in its wide phase."""
        b, f, r, w = _c_i64(), _c_i64(), _c_i64(), _c_i64()
        _check(self._lib.rr_screen_counts(self._h, ctypes.byref(b), ctypes.byref(f), ctypes.byref(r),
                                          ctypes.byref(w)))
        return b.value, f.value, r.value, w.value

    def screen_state(self) -> Tuple[bool, int, int]:
        """(full per-lane lists in use, search blocks still paused to the exact kernel, pauses so far)."""
        f, p, n = _c_i32(), _c_i64(), _c_i64()
        _check(self._lib.rr_screen_state(self._h, ctypes.byref(f), ctypes.byref(p), ctypes.byref(n)))
        return bool(f.value), p.value, n.value

    def set_option(self, name: str, value: int) -> None:
        """A path setting (rr_set_option: screen_grid, verify_cus, x_slots, x_exchange_delay_us, x_host_wait_us,
        x_thread, wide_verify, screen_ct8, screen_i8_pieces, screen_guided, screen_full_lists, screen_i8_min_rows).
        Results are the same under every value."""
        _check(self._lib.rr_set_option(self._h, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = _c_i64()
        _check(self._lib.rr_get_option(self._h, name.encode(), ctypes.byref(v)))
        return v.value

    def screen_factors(self, row_begin: int, n_rows: int, int8: bool = True):
        """(norms, int8 scales, int8 error norms) of rows [row_begin, row_begin + n_rows): the per-row factors the
        screens read (the last two None when int8 is False)."""
        nrm = np.empty(n_rows, dtype=np.float32)
        sc = np.empty(n_rows, dtype=np.float32) if int8 else None
        er = np.empty(n_rows, dtype=np.float32) if int8 else None
        _check(self._lib.rr_screen_factors(self._h, row_begin, n_rows, _fptr(nrm), _fptr(sc) if int8 else None,
                                           _fptr(er) if int8 else None))
        return nrm, sc, er

    def set_timeout(self, ms: int) -> None:
        """Deadline of every host wait on device work, both modes (0 = unbounded); a miss raises
        HipRetrievalError with code RR_E_TIMEOUT (naming the rank or shard, device and stream) and fails
        the handle."""
        _check(self._lib.rr_set_timeout(self._h, int(ms)))

    def stream_queues(self, shard: int = 0) -> list:
        """Hardware-queue addresses of local shard `shard`'s five streams (compute 0, compute 1, exchange
        lanes 0 and 1, staging); equal addresses share one in-order queue (diagnostic)."""
        out = (ctypes.c_uint64 * 5)()
        _check(self._lib.rr_stream_queues(self._h, int(shard), out))
        return list(out)

    def set_timing(self, enable: bool) -> None:
        _check(self._lib.rr_set_timing(self._h, 1 if enable else 0))

    def kernel_time(self, reset: bool = True) -> Tuple[float, int]:
        ms, cnt = ctypes.c_double(), _c_i64()
        _check(self._lib.rr_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(cnt), 1 if reset else 0))
        return ms.value, cnt.value
