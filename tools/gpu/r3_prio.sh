#!/bin/bash
# Round 3: static priority for waves 4-7 (new) vs 58912a7 (base): A/B on the config-5 shard, the 8-GPU shard and
# the headline.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab_prio.txt &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_prio.txt "6250000 64 10 bf16" new base &&
REPS=3 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_prio.txt "125000 32 5 fp32" new base &&
REPS=3 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_prio.txt "1000000 32 5 fp32" new base
