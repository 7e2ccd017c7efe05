#!/bin/bash
# A/B of the working tree against a previous commit on one GPU box, interleaved in one call.
# Prepare (CPU side): git worktree add ab_prev <commit> && make -C ab_prev/rag-serving-system_amd
# Run:  gpurun -- 'bash tools/ab_prev.sh > gpurun_out/ab.log 2>&1'     Clean up: git worktree remove ab_prev
set -e
r() { (cd "$1" && timeout -k 10 120 python bench.py --steps 300 --no-cpu-baseline --no-pmc --variants "" \
        --ingest-rows 0 --latency-steps 20 $2 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 $2', d['ms_per_step'], d['roofline']['kernel_avg_us'])"); }
for i in 1 2; do r ab_prev; r . ; r ab_prev "--docs 125000"; r . "--docs 125000"; done
