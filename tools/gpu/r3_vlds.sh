#!/bin/bash
# Round 3: verify lists prefetched into LDS by LDS-DMA (new) vs HEAD (base): screen/config tests, A/B at the 8-/4-GPU
# shard sizes and the headline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_configs.py > gpurun_out/t_vlds.log 2>&1 &&
rm -f gpurun_out/ab_vlds.txt &&
REPS=3 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_vlds.txt "125000 32 5 fp32" new base &&
REPS=2 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_vlds.txt "250000 32 5 fp32" new base &&
REPS=2 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_vlds.txt "1000000 32 5 fp32" new base
