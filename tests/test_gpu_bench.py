"""bench.py on the GPU at a small size, through both data paths the driver's runs take: one shard (N = 1) and the
multi-GPU path (a 1-rank RCCL communicator: every search block all-gathered over the exchange lanes and merged on
the device, as each rank of an N-GPU run does). The line must carry the contract's fields and a consistent
roofline; results of the exchange path are checked against the oracle in test_gpu_api / test_gpu_screen."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("exchange", [False, True])
def test_bench_line(hip, exchange):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--docs", "40000", "--steps", "12",
           "--warmup", "3", "--latency-steps", "4", "--steady-steps", "12", "--no-cpu-baseline", "--variants", "",
           "--ingest-rows", "0", "--no-pmc"] + (["--exchange-1rank"] if exchange else [])
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in rec, key
    r = rec["roofline"]
    assert rec["value"] > 0 and rec["n_gpus"] == 1 and rec["steps"] == 12
    assert r["compute_streams"] == 2 and r["kernel_le_step"]
    assert r["screen_fallbacks"] == 0 and r["screened_blocks"] > 0
    assert r["kernel_alone"] and r["kernel_alone"]["launches"] == 40
    assert rec["rccl_ranks"] == (1 if exchange else 0)
    assert rec["exchange"].startswith("rccl") == exchange
