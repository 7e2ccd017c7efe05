#!/bin/bash
# Round 3: epilogue one tile late (MFMA shadow): full GPU suite, then A/B vs ccee35d (config-5 shard, headline).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_pipe.log 2>&1 &&
rm -f gpurun_out/ab_pipe.txt &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_pipe.txt "6250000 64 10 bf16" new r3g &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_pipe.txt "1000000 32 5 fp32" new r3g
