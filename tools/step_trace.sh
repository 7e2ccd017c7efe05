#!/bin/bash
# Kernel + memory-copy trace of one bench workload (run inside gpurun), for per-step gap analysis.
#   bash tools/step_trace.sh gpurun_out/<dir> <docs> [k]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/t" -o t --output-format csv -- \
  python3 "$R/bench.py" --gpus 1 --docs $2 --k ${3:-5} --steps 200 --warmup 20 --latency-steps 5 --steady-steps 50 \
  --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc > "$O/bench.json" 2> "$O/err.txt"
