"""In-process request queue with time/size-bounded batch formation — the retriever's caller side
(SURVEY.md §8(f) row 4).

Mirrors the interface and batching rule of the reference's in-memory ``RequestQueue``
(``rag_service/core/request_queue.py:82-135``): ``add_request`` / ``get_batch`` / ``store_result`` /
``get_result``. The batching rule decides serving latency, so it is kept exactly:

* a batch closes when it holds ``max_batch_size`` requests;
* or, once it holds at least one request, when ``max_wait_time`` has passed since ``get_batch`` began;
* or when one wait for the next request times out. Each wait lasts the time left of ``max_wait_time``
  but never less than 0.1 s (:112), so an idle queue returns an empty batch after ``max_wait_time``
  (0.1 s at least), and a non-empty batch closes at most 0.1 s after the window ends.

``on_result`` (not in the reference) is called with the request id whenever a result is stored, so a
replay harness can time completion without polling.
"""
from __future__ import annotations

import queue
import threading
import time
import uuid
from typing import Any, Callable, Optional


class RequestQueue:
    def __init__(self, max_batch_size: int = 8, max_wait_time: float = 0.5, polling_interval: float = 0.1,
                 on_result: Optional[Callable[[str], None]] = None):
        self.queue: "queue.Queue[dict]" = queue.Queue()
        self.results: dict = {}
        self.max_batch_size = max_batch_size
        self.max_wait_time = max_wait_time
        self.polling_interval = polling_interval
        self.lock = threading.Lock()
        self.on_result = on_result

    def add_request(self, query: str, k: int = 2, request_id: Optional[str] = None) -> str:
        rid = request_id or str(uuid.uuid4())
        self.queue.put({"id": rid, "query": query, "k": k})
        return rid

    def get_batch(self) -> list:
        batch = []
        t0 = time.time()
        while len(batch) < self.max_batch_size:
            waited = time.time() - t0
            if batch and waited >= self.max_wait_time:
                break
            try:
                batch.append(self.queue.get(timeout=max(0.1, self.max_wait_time - waited)))
                self.queue.task_done()
            except queue.Empty:
                break
        return batch

    def store_result(self, request_id: str, result: Any):
        with self.lock:
            self.results[request_id] = result
        if self.on_result is not None:
            self.on_result(request_id)

    def get_result(self, request_id: str, timeout: float = 30) -> Optional[Any]:
        deadline = time.time() + timeout
        while time.time() < deadline:
            with self.lock:
                if request_id in self.results:
                    return self.results.pop(request_id)
            time.sleep(self.polling_interval)
        return None
