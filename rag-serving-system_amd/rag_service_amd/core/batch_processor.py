"""BatchProcessor drop-in whose retrieval step runs on the MI355X retriever.

Mirrors the reference's ``rag_service/core/batch_processor.py`` (BatchProcessor, :15-125): same
constructor signature and thread loop, same embedding semantics (the retrieval hot path's caller,
SURVEY.md §8a row a8), same result/error conventions. Differences, all on the retrieval hand-off:

* the query embeddings stay on the GPU: when the retriever exposes ``batch_retrieve_device`` (the HIP
  retrievers do) the (B, 1024) fp32 tensor's device pointer is handed to the C-ABI
  (``rr_set_queries_device``) instead of the reference's ``.cpu().numpy()`` round trip (:92);
  ``device_handoff=False`` restores the host path;
* the LLM prompt list is passed directly (the reference wraps it in ``datasets.Dataset`` only to read
  the same list back, :104-105).

The embedding half (e5 forward) is PyTorch-ROCm, as BASELINE config 4 specifies; its semantics are kept
exactly: "query: " prefix, tokenizer(padding=True, truncation=True), ``last_hidden_state.mean(dim=1)``
over ALL positions (pad tokens included, no attention-mask weighting) and no L2 normalisation
(:83-91).
"""
from __future__ import annotations

import logging
import threading
import time
from typing import List

logger = logging.getLogger(__name__)


def embed_queries(embedding_model: dict, queries: List[str], device):
    """batch_processor.py:82-91 — returns the (B, H) fp32 tensor on `device`."""
    import torch
    with torch.no_grad():
        inputs = [f"query: {query}" for query in queries]
        encoded = embedding_model["tokenizer"](inputs, padding=True, truncation=True, return_tensors="pt")
        encoded = {k: v.to(device) for k, v in encoded.items()}
        outputs = embedding_model["model"](**encoded)
        return outputs.last_hidden_state.mean(dim=1)


class BatchProcessor(threading.Thread):
    """Background thread that processes batches of RAG requests (batch_processor.py:15-125)."""

    def __init__(self, request_queue, embedding_model: dict, llm_model, retriever, device: str = "cuda",
                 polling_interval: float = 0.1, device_handoff: bool = True):
        super().__init__(daemon=True)
        import torch
        self.request_queue = request_queue
        self.embedding_model = embedding_model
        self.llm_model = llm_model
        self.retriever = retriever
        self.device = torch.device(device)
        self.polling_interval = polling_interval
        self.device_handoff = device_handoff
        self.running = True
        try:
            self.embedding_model["model"].to(self.device)
            logger.info("embedding model placed on %s", self.device)
        except Exception as e:
            logger.error("could not place the embedding model on %s: %s", self.device, e)
        logger.info("batch processor ready")

    def stop(self):
        logger.info("batch processor stopping")
        self.running = False

    # batch_processor.py:47-71
    def run(self):
        logger.info("batch processor running")
        while self.running:
            try:
                batch = self.request_queue.get_batch()
                if not batch:
                    time.sleep(self.polling_interval)
                    continue
                logger.info("batch of %d requests", len(batch))
                start_time = time.time()
                self._process_batch(batch)
                logger.info("batch done in %.4f s", time.time() - start_time)
            except Exception as e:
                logger.error("run loop: unexpected failure, continuing: %s", e, exc_info=True)
        logger.info("batch processor stopped")

    def retrieve(self, queries: List[str], ks: List[int]) -> List[List[str]]:
        """Embedding half + retrieval (the path BASELINE config 4 measures end to end)."""
        import torch
        emb = embed_queries(self.embedding_model, queries, self.device)
        # the C-ABI reads a device pointer on the retriever's FIRST device; any other placement takes the host path
        first = getattr(self.retriever, "devices", [0])[0]
        if (self.device_handoff and emb.is_cuda and emb.device.index == first
                and hasattr(self.retriever, "batch_retrieve_device")):
            emb = emb.float().contiguous()
            torch.cuda.current_stream(emb.device).synchronize()   # the C-ABI reads it on its own stream
            out = self.retriever.batch_retrieve_device(emb.data_ptr(), emb.shape[0], emb.shape[1], ks)
            del emb
            return out
        return self.retriever.batch_retrieve(emb.cpu().numpy(), ks)

    # batch_processor.py:74-125
    def _process_batch(self, batch):
        request_ids = [req["id"] for req in batch]
        try:
            queries = [req["query"] for req in batch]
            ks = [req["k"] for req in batch]
            all_retrieved_docs = self.retrieve(queries, ks)
            all_contexts = ["\n---\n".join(docs) for docs in all_retrieved_docs]
            prompts = [f"Context:\n{c}\n\nQuestion: {q}\n\nThe Answer to this question is: "
                       for q, c in zip(queries, all_contexts)]
            outputs = self.llm_model(prompts, max_new_tokens=10, do_sample=True, batch_size=len(prompts))
            for i, request_id in enumerate(request_ids):
                try:
                    self.request_queue.store_result(request_id, {"result": str(outputs[i])})
                except Exception as e:
                    logger.error("request %s: storing its result failed: %s", request_id, e)
                    self.request_queue.store_result(request_id, {"error": str(e)})
        except Exception as e:
            logger.error("batch of %d requests failed: %s", len(request_ids), e)
            for request_id in request_ids:
                self.request_queue.store_result(request_id, {"error": str(e), "status": "failed"})
