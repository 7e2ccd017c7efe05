"""Serving-level replay: request arrivals from the reference's load-generator traces, batched by the
reference's time/size rule, served by ``BatchProcessor`` + the HIP retriever, with the reference's
latency summary.

Reference pieces restated here:

* ``generate_trace`` — ``benchmarks/load_generator.py:19-54``: request send times in ms for the
  "uniform", "poisson" and "random" patterns, from NumPy's legacy Mersenne-Twister stream seeded like
  ``np.random.seed(seed)`` (bit-identical timestamps; pinned by tests/golden/golden_serving.json).
* ``latency_summary`` — ``benchmarks/metrics/collector.py:34-69``: request counts, throughput over the
  whole run, latency min / max / mean / p50 / p95 / p99 (``np.percentile``, linear).
* batch formation — ``core.request_queue.RequestQueue`` (``request_queue.py:99-118``).

The replay runs in one process with no HTTP: a dispatcher thread releases each request at its trace time
into the queue (where the reference's client POSTs ``/rag``), the reference-shaped ``BatchProcessor``
thread forms batches, embeds, retrieves and stores results, and a request's latency runs from its release
to the moment its result is stored. The reference's client finds results by polling ``/rag/result`` every
``polling_interval`` (``load_generator.py:91-116``), which adds up to one interval; ``client_poll``
reports that quantised figure too. The LLM step is out of scope; the stand-in returns the
prompt it was given, so each result carries the retrieved context and can be checked.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

from .core.request_queue import RequestQueue


def generate_trace(pattern: str, rps: int, duration: int, seed: Optional[int] = None) -> List[int]:
    total = rps * duration
    horizon = duration * 1000
    if total == 0:
        return []
    rng = np.random.RandomState(seed)        # np.random.seed(seed) + the module functions: the same stream
    if pattern == "uniform":
        step = horizon / total
        t = np.concatenate([[0.0], np.cumsum(np.full(total - 1, step))])   # sequential sums, as the loop
        out = np.minimum(np.rint(t).astype(np.int64), horizon - 1)
    elif pattern == "poisson":
        gaps = rng.exponential(1 / (rps / 1000), total)
        t = np.concatenate([[0.0], np.cumsum(gaps[:-1])])
        out = np.rint(t).astype(np.int64)
        out = out[out < horizon]
    elif pattern == "random":
        out = rng.randint(0, horizon, size=total)
    else:
        raise ValueError(f"unknown trace pattern {pattern!r}")
    return sorted(int(v) for v in out)


def latency_summary(latencies: Sequence[float], success: int, errors: int, total_time: float) -> Dict:
    n = success + errors
    out = {"total_requests": n, "successful_requests": success, "failed_requests": errors,
           "total_time": total_time,
           "throughput": n / total_time if total_time > 0 else 0,
           "throughput_successful": success / total_time if total_time > 0 else 0}
    if len(latencies):
        lat = list(latencies)
        out["latency"] = {"min": min(lat), "max": max(lat), "mean": sum(lat) / len(lat),
                          **{f"p{p}": float(np.percentile(lat, p)) for p in (50, 95, 99)}}
    else:
        out["latency"] = {key: 0 for key in ("min", "max", "mean", "p50", "p95", "p99")}
    return out


class EmbeddingTable:
    """Embedding-model stand-in for retrieval-only serving: query i's embedding is row i of a table kept on
    the device. ``tokenizer`` maps each "query: <text>" to its row, ``model`` gathers the rows as a
    (B, 1, H) hidden state, so ``embed_queries``' mean over positions returns them unchanged."""

    def __init__(self, texts: Sequence[str], table, device):
        import torch
        self.row = {f"query: {t}": i for i, t in enumerate(texts)}
        self.table = torch.as_tensor(np.ascontiguousarray(table, dtype=np.float32), device=device)
        tab = self.table

        class _Out:
            def __init__(self, h):
                self.last_hidden_state = h

        class _Model:
            def to(self, dev):
                return self

            def __call__(self, input_ids, **_):
                return _Out(tab[input_ids.to(tab.device)])

        def tokenizer(inputs, padding=True, truncation=True, return_tensors="pt"):
            return {"input_ids": torch.tensor([[self.row[s]] for s in inputs])}

        self.model = {"tokenizer": tokenizer, "model": _Model()}


def echo_llm(prompts, max_new_tokens=10, do_sample=True, batch_size=None):
    """LLM stand-in: returns each prompt (generation is out of scope)."""
    return list(prompts)


def replay(processor_cls, retriever, embedding_model, texts: Sequence[str], trace_ms: Sequence[int], k: int = 2,
           max_batch_size: int = 32, max_wait_time: float = 1.0, polling_interval: float = 0.3,
           processor_poll: float = 0.1, device: str = "cuda", timeout: float = 120.0,
           keep_results: bool = False) -> Dict:
    """Serve len(trace_ms) requests (request i asks texts[i % len(texts)]) released at trace_ms[i].
    Defaults are the reference service's: Settings max_batch_size 32, max_wait_time 1.0 s, polling_interval
    0.3 s (config.py:8-10; the client's poll period), the BatchProcessor's idle sleep 0.1 s (its default,
    main.py:58-64), k = 2 (the HTTP default, api/models.py:6)."""
    n = len(trace_ms)
    start = np.zeros(n)
    end = np.full(n, np.nan)
    done = threading.Event()
    remaining = [n]
    lock = threading.Lock()
    batch_sizes: List[int] = []

    def on_result(rid: str):
        i = int(rid)
        end[i] = time.perf_counter()
        with lock:
            remaining[0] -= 1
            if remaining[0] == 0:
                done.set()

    q = RequestQueue(max_batch_size=max_batch_size, max_wait_time=max_wait_time,
                     polling_interval=polling_interval, on_result=on_result)
    get_batch = q.get_batch

    def counting_get_batch():
        b = get_batch()
        if b:
            batch_sizes.append(len(b))
        return b

    q.get_batch = counting_get_batch
    proc = processor_cls(q, embedding_model, echo_llm, retriever, device=device, polling_interval=processor_poll)
    proc.start()
    t0 = time.perf_counter()
    for i, ms in enumerate(trace_ms):
        wait = t0 + ms / 1000.0 - time.perf_counter()
        if wait > 0:
            time.sleep(wait)
        start[i] = time.perf_counter()
        q.add_request(texts[i % len(texts)], k, request_id=str(i))
    if n:
        done.wait(timeout)
    total_time = time.perf_counter() - t0
    proc.stop()
    proc.join(timeout=max_wait_time + 5)
    results = {i: q.results.get(str(i)) for i in range(n)}
    ok = ~np.isnan(end)                                       # a result (answer or error) was stored
    failed = sum(1 for i in range(n) if results[i] is None or "error" in results[i])
    lat = (end - start)[ok]
    out = latency_summary(lat.tolist(), n - failed, failed, total_time)
    poll = np.ceil(lat / polling_interval) * polling_interval if polling_interval > 0 else lat
    out["client_poll"] = {f"p{p}": float(np.percentile(poll, p)) for p in (50, 95, 99)} if len(lat) else {}
    out["batches"] = len(batch_sizes)
    out["mean_batch"] = float(np.mean(batch_sizes)) if batch_sizes else 0.0
    if keep_results:
        out["results"] = results
    return out


def context_docs(result: Dict) -> List[str]:
    """The retrieved documents inside an ``echo_llm`` result (the prompt of batch_processor.py:103)."""
    text = result["result"]
    ctx = text[len("Context:\n"):text.index("\n\nQuestion: ")]
    return ctx.split("\n---\n") if ctx else []
