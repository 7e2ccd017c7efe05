#!/bin/bash
# Round 3: epilogue without rcp (fma bar), vector factor reads, packed partial sums (new) vs the stagger alone (stg) vs HEAD (base)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_epi.log 2>&1 &&
rm -f gpurun_out/ab_epi.txt &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_epi.txt "6250000 64 10 bf16" new base stg &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_epi.txt "1000000 32 5 fp32" new base stg &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_epi.txt "125000 32 5 fp32" new base stg &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_epi.txt "1000000 32 5 bf16" new base
