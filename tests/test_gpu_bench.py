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


def test_bench_replica_groups_on_one_gpu(hip):
    """The N > 1 placement path (R replica groups) end to end: two ranks launched the driver's way (`--gpus 2` spawns
    torch.distributed.run), both on cuda:0 (test hook --same-device), each a whole-corpus replica with a 1-rank RCCL
    exchange searching its own batches; rank 0's line counts both groups' batches (parallelism and scaling say so).
    The groups' 2-rank communicators need distinct GPUs and are not reachable on a one-GPU box."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--same-device", "--shard-group", "1",
           "--exchange-1rank", "--no-row-shard-all", "--docs", "70000", "--steps", "12", "--warmup", "3",
           "--latency-steps", "4", "--steady-steps", "12", "--no-cpu-baseline", "--variants", "", "--ingest-rows", "0",
           "--no-pmc"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=REPO, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(recs) == 1, out.stdout[-2000:]
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["scaling"] == "weak"
    assert rec["placement"]["shard_group"] == 1 and rec["placement"]["replica_groups"] == 2
    assert rec["config"]["parallelism"] == "row-shard x1, replica groups x2"
    assert rec["rccl_ranks"] == 1 and rec["row_shard_all"] is None
    assert rec["roofline"]["screen_fallbacks"] == 0
