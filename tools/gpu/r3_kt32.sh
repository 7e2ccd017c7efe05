#!/bin/bash
# Round 3: the large-k path (k = 64, 32-entry lists + wide output) at this head (new: immediate inserts for 32-entry
# lists), without the stagger (nostg), without the priority (noprio), and the session's start 33f7f7c (s0).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab_kt32b.txt
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_kt32b.txt "1000000 32 64 fp32" new nostg noprio s0 &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_kt32b.txt "1000000 32 20 bf16" new nostg s0
