"""Drop-in retrievers backed by the MI355X C-ABI (librag_retrieval.so).

Two classes mirror the reference's two live retrievers (ngray0/RAG-Serving-System,
rag_service/core/retriever.py), keeping their constructor, method names, argument meaning,
validation order, k-clamping and "log and return empty lists" error convention:

* ``HipRetriever``        <- ``CupyRetriever``   (retriever.py:564-799): clipped cosine similarity,
                             strict ``isinstance(k, int)`` check, ``max_k`` batching + per-query slicing.
                             This is the class ``main.py:52-55`` / ``batch_processor.py:11,21`` use.
* ``HipSimpleRetriever``  <- ``SimpleRetriever`` (retriever.py:57-166): raw dot product, per-query k
                             rules of ``retrieve`` applied to every query of a batch.

All arithmetic happens in the HIP kernels; there is no NumPy/CPU fallback. If the extension is missing,
construction raises ``HipRetrievalUnavailable``.

Deliberate, documented difference: ties between exactly equal scores are broken by ascending document
index (the reference's order on ties is whatever numpy introselect / CuPy's sort produce).
"""
from __future__ import annotations

import logging
import numbers
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .._lib import Index

logger = logging.getLogger(__name__)


def _is_integral(k) -> bool:
    return isinstance(k, (numbers.Integral, np.integer))


class _HipRetrieverBase:
    _metric = "cosine"

    def __init__(self, doc_embeddings: np.ndarray, documents: List[str], dtype: str = "fp32",
                 devices: Optional[Sequence[int]] = None):
        if doc_embeddings.dtype != np.float32:
            logger.warning("corpus arrives as %s; storing float32 values", doc_embeddings.dtype)
            doc_embeddings = doc_embeddings.astype(np.float32)
        try:
            self.index = Index(devices=devices, dtype=dtype, metric=self._metric)
            self.index.load(doc_embeddings)
            logger.info("corpus %s resident in HBM: storage %s, metric %s, devices %s", doc_embeddings.shape, dtype,
                        self._metric, list(devices) if devices else [0])
        except Exception as e:
            logger.error("corpus upload to the GPU failed: %s", e, exc_info=True)
            raise
        self.documents = documents
        self.devices = list(devices) if devices else [0]
        self.N_A = int(doc_embeddings.shape[0])
        self.D = int(doc_embeddings.shape[1])
        self.dtype = dtype

    # extra (not in the reference): raw device results for tests and benchmarks
    def search(self, queries: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        """(scores [b,k] fp32, global indices [b,k] int64) sorted by (score desc, index asc)."""
        return self.index.search(np.atleast_2d(np.asarray(queries, dtype=np.float32)), int(k))

    def search_device(self, dev_ptr: int, batch_size: int, dim: int, k: int) -> Tuple[np.ndarray, np.ndarray]:
        """Like search(), for a (batch_size, dim) row-major fp32 buffer already in HBM on the retriever's
        first device (device-to-device copy into the C-ABI, rr_set_queries_device)."""
        self.index.set_queries_device(int(dev_ptr), int(batch_size), int(dim))
        self.index.search_staged(int(k))
        return self.index.fetch()

    def _docs(self, idx_row: np.ndarray, k_i: int) -> List[str]:
        valid = idx_row[idx_row >= 0][:k_i]
        return [self.documents[int(j)] for j in valid]

    def close(self) -> None:
        self.index.close()


class HipRetriever(_HipRetrieverBase):
    """Drop-in for ``CupyRetriever`` (retriever.py:564-799): clipped cosine similarity on MI355X."""

    _metric = "cosine"

    def __init__(self, doc_embeddings: np.ndarray, documents: List[str], dtype: str = "fp32",
                 devices: Optional[Sequence[int]] = None, metric: str = "cosine"):
        self._metric = metric
        super().__init__(doc_embeddings, documents, dtype=dtype, devices=devices)
        logger.info("HipRetriever ready: %d rows x %d", self.N_A, self.D)

    # retriever.py:615-683
    def retrieve(self, query_emb: np.ndarray, k: int = 2) -> List[str]:
        start_time = time.time()
        if not isinstance(query_emb, np.ndarray):
            logger.error("retrieve: query must be a numpy.ndarray, not %s", type(query_emb).__name__)
            return []
        if query_emb.ndim == 2 and query_emb.shape[0] == 1:
            query_emb = query_emb.flatten()
        elif query_emb.ndim != 1:
            logger.error("retrieve: query shape %s is neither (dim,) nor (1, dim)", query_emb.shape)
            return []
        if query_emb.shape[0] != self.D:
            logger.error("retrieve: query has %d dimensions, the corpus %d", query_emb.shape[0], self.D)
            return []
        actual_k = min(k, self.N_A)
        if actual_k <= 0:
            logger.warning("retrieve: k=%s leaves nothing to return", k)
            return []
        try:
            if not _is_integral(actual_k):
                raise TypeError(f"k must be an integer, got {type(k)}")
            if query_emb.dtype != np.float32:
                query_emb = query_emb.astype(np.float32)
            _, idx = self.index.search(query_emb.reshape(1, self.D), int(actual_k))
            docs = self._docs(idx[0], int(actual_k))
            logger.debug("retrieve: %.6f s", time.time() - start_time)
            return docs
        except Exception as e:
            logger.error("retrieve failed: %s", e, exc_info=True)
            return []

    # retriever.py:686-799
    def batch_retrieve(self, query_embeddings: np.ndarray, ks: List[int]) -> List[List[str]]:
        start_time = time.time()
        batch_size = query_embeddings.shape[0]   # read before the type check, as the reference does (:702)

        if not isinstance(query_embeddings, np.ndarray):
            logger.error("batch_retrieve: queries must be a numpy.ndarray, not %s", type(query_embeddings).__name__)
            return [[] for _ in ks]
        if query_embeddings.ndim != 2:
            logger.error("batch_retrieve: queries must be 2-D, got %d-D", query_embeddings.ndim)
            return [[] for _ in ks]
        if batch_size == 0:
            logger.info("batch_retrieve: empty batch")
            return []
        if not isinstance(ks, list) or batch_size != len(ks):
            logger.error("batch_retrieve: %d queries but %d k values", batch_size, len(ks))
            return [[] for _ in range(batch_size)]
        if query_embeddings.shape[1] != self.D:
            logger.error("batch_retrieve: queries have %d dimensions, the corpus %d", query_embeddings.shape[1], self.D)
            return [[] for _ in ks]
        if not all(isinstance(k_val, int) for k_val in ks):
            logger.error("batch_retrieve: every k must be a Python int")
            return [[] for _ in ks]

        valid_ks = [k_val for k_val in ks if k_val > 0]
        if not valid_ks:
            logger.warning("batch_retrieve: no positive k in the batch")
            return [[] for _ in ks]
        max_k = min(max(valid_ks), self.N_A)
        if max_k <= 0:
            return [[] for _ in ks]

        try:
            if query_embeddings.dtype != np.float32:
                query_embeddings = query_embeddings.astype(np.float32)
            _, idx = self.index.search(query_embeddings, int(max_k))
            batch_results = []
            for i in range(batch_size):
                k_i = ks[i]
                if k_i <= 0:
                    batch_results.append([])
                    continue
                batch_results.append(self._docs(idx[i], k_i))
            logger.debug("batch_retrieve: %.6f s", time.time() - start_time)
            return batch_results
        except Exception as e:
            logger.error("batch_retrieve failed: %s", e, exc_info=True)
            return [[] for _ in ks]


    def batch_retrieve_device(self, dev_ptr: int, batch_size: int, dim: int, ks: List[int]) -> List[List[str]]:
        """batch_retrieve() for query embeddings that are already on the GPU: a (batch_size, dim) fp32
        row-major device buffer, fully written (the caller has synchronised its producing stream).
        Same validation, k rules and results as batch_retrieve; skips the .cpu().numpy() round trip
        of batch_processor.py:92."""
        if batch_size == 0:
            return []
        if not isinstance(ks, list) or batch_size != len(ks):
            logger.error("batch_retrieve: %d queries but %d k values", batch_size, len(ks))
            return [[] for _ in range(batch_size)]
        if dim != self.D:
            logger.error("batch_retrieve_device: queries have %d dimensions, the corpus %d", dim, self.D)
            return [[] for _ in ks]
        if not all(isinstance(k_val, int) for k_val in ks):
            logger.error("batch_retrieve: every k must be a Python int")
            return [[] for _ in ks]
        valid_ks = [k_val for k_val in ks if k_val > 0]
        if not valid_ks:
            return [[] for _ in ks]
        max_k = min(max(valid_ks), self.N_A)
        try:
            _, idx = self.search_device(dev_ptr, batch_size, dim, max_k)
            return [[] if ks[i] <= 0 else self._docs(idx[i], ks[i]) for i in range(batch_size)]
        except Exception as e:
            logger.error("batch_retrieve_device failed: %s", e, exc_info=True)
            return [[] for _ in ks]


class HipSimpleRetriever(_HipRetrieverBase):
    """Drop-in for ``SimpleRetriever`` (retriever.py:57-166): raw dot-product similarity on MI355X."""

    _metric = "dot"

    def __init__(self, doc_embeddings: np.ndarray, documents: List[str], dtype: str = "fp32",
                 devices: Optional[Sequence[int]] = None):
        super().__init__(doc_embeddings, documents, dtype=dtype, devices=devices)
        logger.info("HipSimpleRetriever ready: %d documents", len(self.documents))

    # per-query k rules of retrieve (:89-94): None -> invalid, else the clamped k
    def _effective_k(self, k) -> Optional[int]:
        if k <= 0:
            return None
        if k > self.N_A:
            k = self.N_A
        return int(k) if _is_integral(k) else None

    # retriever.py:78-128
    def retrieve(self, query_emb: np.ndarray, k: int = 2) -> List[str]:
        if k <= 0:
            logger.warning("retrieve: k=%s is not positive", k)
            return []
        if k > self.N_A:
            logger.warning("retrieve: k=%s exceeds the %d documents; returning all of them", k, self.N_A)
            k = self.N_A
        try:
            if query_emb.dtype != np.float32:
                query_emb = query_emb.astype(np.float32)
            if query_emb.ndim != 1:
                if query_emb.ndim == 2 and query_emb.shape[0] == 1:
                    query_emb = query_emb.flatten()
                else:
                    logger.error("retrieve: query shape %s is not 1-D", query_emb.shape)
                    return []
            if query_emb.shape[0] != self.D:
                logger.error("retrieve: query has %d dimensions, the corpus %d", query_emb.shape[0], self.D)
                return []
            if not _is_integral(k):
                raise TypeError(f"k must be an integer, got {type(k)}")
            _, idx = self.index.search(query_emb.reshape(1, self.D), int(k))
            return self._docs(idx[0], int(k))
        except Exception as e:
            logger.error("retrieve failed: %s", e, exc_info=True)
            return []

    # retriever.py:131-166 — same per-query results as calling retrieve() B times, one device pass
    def batch_retrieve(self, query_embeddings: np.ndarray, ks: List[int]) -> List[List[str]]:
        if query_embeddings.ndim != 2:
            logger.error("batch_retrieve: queries must be 2-D, got %d-D", query_embeddings.ndim)
            return [[] for _ in ks]
        if query_embeddings.shape[0] != len(ks):
            logger.error("batch_retrieve: %d queries but %d k values", query_embeddings.shape[0], len(ks))
            return [[] for _ in ks]
        if query_embeddings.shape[1] != self.D:
            logger.error("batch_retrieve: queries have %d dimensions, the corpus %d", query_embeddings.shape[1], self.D)
            return [[] for _ in ks]

        eff = [self._effective_k(k) for k in ks]
        results: List[List[str]] = [[] for _ in ks]
        rows = [i for i, e in enumerate(eff) if e is not None]
        if not rows:
            return results
        try:
            q = query_embeddings[rows]
            if q.dtype != np.float32:
                q = q.astype(np.float32)
            _, idx = self.index.search(q, max(eff[i] for i in rows))
            for j, i in enumerate(rows):
                results[i] = self._docs(idx[j], eff[i])
            return results
        except Exception as e:
            logger.error("batch_retrieve failed: %s", e, exc_info=True)
            return [[] for _ in ks]


# Names a maintainer can import in place of the reference's classes.
CupyRetriever = HipRetriever
SimpleRetriever = HipSimpleRetriever
