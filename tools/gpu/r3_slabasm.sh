#!/bin/bash
# Round 3: a whole slab per inline-asm statement (one lgkmcnt wait and one M0 save/restore per slab, per-lane row
# offsets) (slab, tools/ab build) vs the in-tree default (new): full GPU suite, then A/B on the headline, the 8-GPU shard and config 5's shard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
RR_LIBRARY=$GRAFT_REPO_ROOT/tools/ab/librag_retrieval_slab.so timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_slab.log 2>&1 &&
rm -f gpurun_out/ab_slab.txt &&
REPS=3 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_slab.txt "1000000 32 5 fp32" slab new &&
REPS=3 STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_slab.txt "125000 32 5 fp32" slab new &&
STEPS=20 WARMUP=5 bash tools/ab/ab.sh gpurun_out/ab_slab.txt "6250000 64 10 bf16" slab new
