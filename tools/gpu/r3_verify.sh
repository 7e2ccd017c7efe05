#!/bin/bash
# Round 3: verify list merge (wave maxima instead of LDS atomics on one address, head ranks over every wave): probe,
# screen GPU tests, A/B vs HEAD at the 8- and 4-GPU shard sizes and 1M.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/vprobe_bin 1000000 > gpurun_out/verify_probe_new.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_screen.py tests/test_gpu_configs.py > gpurun_out/t_verify.log 2>&1 &&
rm -f gpurun_out/ab_verify.txt &&
REPS=4 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_verify.txt "125000 32 5 fp32" new base &&
REPS=3 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_verify.txt "250000 32 5 fp32" new base &&
REPS=3 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_verify.txt "1000000 32 5 fp32" new base
