#!/bin/bash
# Round 3: pipelined K-partial exchange (new) vs the staggered epilogue (stg) vs HEAD (base): screen/config GPU tests, then A/B vs HEAD (config-5 shard,
# headline) with the 64-slot two-slab lookahead as a third arm.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/t_stagger.log 2>&1 &&
rm -f gpurun_out/ab_stagger.txt &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_stagger.txt "6250000 64 10 bf16" new base stg &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_stagger.txt "1000000 32 5 fp32" new base stg &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_stagger.txt "125000 32 5 fp32" new base
