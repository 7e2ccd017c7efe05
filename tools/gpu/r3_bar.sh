#!/bin/bash
# Round 3: tighter exact bar (min over lanes of the J-th entry): full GPU suite, then A/B vs fb7fad9 on the
# headline (+ exact fp32 variant) and config 5's per-GPU shard (6.25M bf16, batch 64, k 10).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_bar.log 2>&1 &&
rm -f gpurun_out/ab_bar.txt &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_bar.txt "6250000 64 10 bf16" new r3f &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_bar.txt "1000000 32 5 fp32" new r3f
