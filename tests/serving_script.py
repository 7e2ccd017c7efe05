"""Scripted arrival plans for the batch-formation parity test (test infrastructure).

`run_plan(queue, arrivals)` starts a consumer thread that calls `queue.get_batch()` in a loop (as the
BatchProcessor does) while the main thread adds request i at arrivals[i] seconds; it returns the batches
as lists of request indices. Decisions in these plans are >= 0.1 s apart, so real-time threads give the
same batches on any lightly loaded host. Used by tests/golden/make_serving_golden.py (on the reference's
RequestQueue) and by tests/test_serving.py (on ours)."""
import threading
import time

# (max_batch_size, max_wait_time, arrival times in s)
PLANS = {
    "burst": (4, 0.5, [0.0] * 10),
    "trickle": (8, 0.5, [0.05, 0.25, 0.40, 0.85, 1.75]),
    "full_then_wait": (3, 0.6, [0.05, 0.06, 0.07, 0.08, 0.3, 1.3]),
    "late_window": (16, 0.3, [0.05, 0.2, 0.5, 0.55, 1.2]),
}


def run_plan(queue, arrivals, settle=0.8):
    batches = []
    stop = threading.Event()

    def consumer():
        while not stop.is_set():
            b = queue.get_batch()
            if b:
                batches.append([int(r["query"]) for r in b])

    th = threading.Thread(target=consumer, daemon=True)
    t0 = time.perf_counter()
    if arrivals and arrivals[0] == 0.0:            # a burst is queued before the consumer starts
        for i, a in enumerate(arrivals):
            if a == 0.0:
                queue.add_request(str(i), 2)
    th.start()
    for i, a in enumerate(arrivals):
        if a == 0.0:
            continue
        w = t0 + a - time.perf_counter()
        if w > 0:
            time.sleep(w)
        queue.add_request(str(i), 2)
    time.sleep(settle)
    stop.set()
    th.join(timeout=5)
    return batches
