#!/bin/bash
# SQ counters: config-5 shard kernel and the fp32 headline screen (two 8-counter passes each).
set -o pipefail
mkdir -p gpurun_out
bash tools/ab/sq_passes.sh gpurun_out/sq_r3/cfg5 "6250000 64 10 bf16" &&
bash tools/ab/sq_passes.sh gpurun_out/sq_r3/fp32 "1000000 32 5 fp32"
