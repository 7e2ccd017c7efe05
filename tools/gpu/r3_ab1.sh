#!/bin/bash
# A/B: screen epilogue rework (new) vs round-3 start (r3a), 1M and 125k rows, fp32 k 5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab_r3_epi.txt
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_r3_epi.txt "1000000 32 5 fp32" new r3a &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_r3_epi.txt "125000 32 5 fp32" new r3a
