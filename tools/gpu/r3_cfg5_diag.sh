#!/bin/bash
# Round 3: decomposition of the 64-slot bf16 pass on config 5's per-GPU shard (tools/kbench_cfg5.hip builds).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/cfg5_diag2.jsonl
for rep in 1 2; do
for D in ${VARIANTS:-d0 d0stg0 d0par d0la2 d1 d1la2 d3 d3stg0 d3la2}; do
  echo "== $D" >> gpurun_out/cfg5_diag2.jsonl
  timeout -k 10 120 tools/kbench_cfg5_$D 6250000 5 >> gpurun_out/cfg5_diag2.jsonl || exit 1
done
done
