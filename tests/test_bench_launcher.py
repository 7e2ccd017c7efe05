"""bench.py as the driver invokes it: `python bench.py --gpus N ...` without torchrun launches one rank per
GPU itself (CPU dry run: gloo control plane only, no GPU call)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 2, 8])
def test_plain_launch_reaches_timed_loop(n):
    """n = 8: the driver's 8-GPU command shape — eight gloo ranks on the CPU."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "20",
                          "--warmup", "5", "--dry-run"], capture_output=True, text=True, timeout=240, env=env,
                         cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["dry_run"] and rec["n_gpus"] == n and rec["ranks_seen"] == n
    assert rec["launched_by"] == ("torch.distributed.run" if n > 1 else "plain")
    # the default placement of 1M docs (auto: row shards of >= 500k rows): pairs of ranks, N / 2 replica groups; every
    # rank received its group's communicator id over the control plane
    pl = rec["placement"]
    assert (pl["shard_group"], pl["replica_groups"]) == ((1, 1) if n == 1 else (2, n // 2))
    assert pl["ranks_with_their_group_id"] == n


@pytest.mark.parametrize("sg,want", [("8", (8, 1)), ("1", (1, 8)), ("3", (4, 2))])
def test_shard_group_option(sg, want):
    """--shard-group S fixes the group size (rounded up to a divisor of N): 8 = the whole node as one row-sharded
    group (the north star's layout), 1 = independent replicas."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--shard-group", sg,
                          "--dry-run"], capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    pl = rec["placement"]
    assert (pl["shard_group"], pl["replica_groups"]) == want and pl["ranks_with_their_group_id"] == 8


def test_placement_rule():
    sys.path.insert(0, os.path.join(REPO, "rag-serving-system_amd"))
    from rag_service_amd.dist import placement
    assert placement(1_000_000, 1) == (1, 1)
    assert placement(1_000_000, 2) == (2, 1)
    assert placement(1_000_000, 4) == (2, 2)
    assert placement(1_000_000, 8) == (2, 4)
    assert placement(10_000_000, 8) == (8, 1)        # config 3: 1.25M-row shards over the whole node
    assert placement(50_000_000, 8) == (8, 1)        # config 5
    assert placement(100_000, 8) == (1, 8)           # a small corpus: replicas
    assert placement(1_500_000, 8) == (4, 2)         # 3 rounded up to a divisor of 8
    assert placement(1_000_000, 8, shard_group=8) == (8, 1)


def test_missed_deadline_exits_loudly():
    """The deadline path of the N > 1 bench: rank 1 stalls past --dist-timeout-s before the
    barrier every rank must pass. Rank 0's wait times out; it prints a JSON error line naming its rank and the
    stage, and exits non-zero (no hang, no re-exec); the launcher's exit status is non-zero."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run",
                          "--dry-run-stall-rank", "1", "--dist-timeout-s", "4"], capture_output=True, text=True,
                         timeout=240, env=env, cwd=REPO)
    assert out.returncode != 0
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    errs = [r for r in recs if r.get("error")]
    assert errs, out.stdout + out.stderr[-2000:]
    r0 = [r for r in errs if r["rank"] == 0]
    assert r0 and r0[0]["stage"] == "dry-run barrier" and r0[0]["value"] is None and r0[0]["n_gpus"] == 2
