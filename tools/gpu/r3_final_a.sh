#!/bin/bash
# Round 3 final evidence, part A: the driver's bench command (PMC child pass, CPU baseline) + rocprofv3 kernel trace
# and stats of the same command; SQ counter passes for the headline screen and the config-5 shard kernel.
set -o pipefail
mkdir -p gpurun_out/r3f
bash tools/prof_round.sh gpurun_out/r3f/driver &&
bash tools/ab/sq_passes.sh gpurun_out/r3f/sq/fp32 "1000000 32 5 fp32" &&
bash tools/ab/sq_passes.sh gpurun_out/r3f/sq/cfg5 "6250000 64 10 bf16"
