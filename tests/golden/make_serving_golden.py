"""Golden vectors for the serving-level pieces, produced by the REFERENCE's own code (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_serving_golden.py

* `generate_trace` of benchmarks/load_generator.py:19-54 for every pattern at several (rps, duration, seed);
* the batches the reference's in-memory RequestQueue (rag_service/core/request_queue.py:82-135) forms
  under the scripted arrival plans of tests/serving_script.py;
* MetricsCollector.calculate_metrics (benchmarks/metrics/collector.py:34-69) on a fixed latency list.

Modules the reference imports that this image lacks get inert stand-ins before the import, as
make_golden.py does for cupy: `pydantic_settings.BaseSettings` (a plain class, so Settings() keeps its
defaults) and `redis` (only RedisRequestQueue, which is not used, touches it). Output:
tests/golden/golden_serving.json (data only).
"""
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(REPO, "tests"), REF, os.path.join(REF, "benchmarks")]

from serving_script import PLANS, run_plan  # noqa: E402


def stand_ins():
    ps = types.ModuleType("pydantic_settings")

    class BaseSettings:
        pass

    ps.BaseSettings = BaseSettings
    sys.modules.setdefault("pydantic_settings", ps)
    rd = types.ModuleType("redis")
    rd.from_url = lambda *a, **k: None
    sys.modules.setdefault("redis", rd)


def main():
    stand_ins()
    import importlib
    lg = importlib.import_module("load_generator")
    rq = importlib.import_module("rag_service.core.request_queue")
    col = importlib.import_module("metrics.collector")
    out = {"traces": [], "batches": {}, "metrics": None}
    for pattern in ("uniform", "poisson", "random"):
        for rps, dur, seed in ((1, 60, 10), (7, 3, 11), (50, 10, 210), (333, 2, 12), (1000, 1, 13), (0, 5, 1)):
            out["traces"].append({"pattern": pattern, "rps": rps, "duration": dur, "seed": seed,
                                  "trace": [int(t) for t in lg.generate_trace(pattern, rps, dur, seed)]})
    for name, (mb, mw, arrivals) in PLANS.items():
        q = rq.RequestQueue(max_batch_size=mb, max_wait_time=mw, polling_interval=0.05)
        out["batches"][name] = run_plan(q, arrivals)
        print(name, out["batches"][name], flush=True)
    mc = col.MetricsCollector()
    mc.latencies = [0.31, 1.2, 0.05, 0.7, 0.7, 2.5, 0.33, 0.9, 1.01, 0.02, 0.4]
    mc.success_count, mc.error_count = 10, 1
    m = mc.calculate_metrics()
    out["metrics"] = {"latencies": mc.latencies, "success": 10, "errors": 1,
                      "latency": {k: float(v) for k, v in m["latency"].items()}}
    with open(os.path.join(HERE, "golden_serving.json"), "w") as f:
        json.dump(out, f)
    print("traces:", len(out["traces"]), "done")


if __name__ == "__main__":
    main()
