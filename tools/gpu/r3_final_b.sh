#!/bin/bash
# Round 3 final evidence, part B: verify-kernel phase probe, then the per-GPU shard sweep of the multi-GPU configs.
set -o pipefail
mkdir -p gpurun_out/r3f
timeout -k 10 120 tools/vprobe_bin 1000000 > gpurun_out/r3f/verify_probe.log 2>&1 &&
true || bash tools/shard_sweep.sh gpurun_out/r3f/shard_sweep.jsonl
