#!/bin/bash
# Round 3 final evidence, part B: per-GPU shard sweep of the multi-GPU configs on one GPU, and the same shards through
# the 1-rank RCCL exchange path.
set -o pipefail
mkdir -p gpurun_out/r3g
bash tools/shard_sweep.sh gpurun_out/r3g/shard_sweep.jsonl &&
bash tools/shard_sweep_x.sh gpurun_out/r3g/shard_sweep_exchange.jsonl
