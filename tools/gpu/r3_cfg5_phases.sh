#!/bin/bash
# Round 3: per-phase cycles of the 64-/32-slot bf16 passes on config 5's per-GPU shard (tools/kbench_cfg5.hip).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/cfg5_phases.jsonl
for D in d4; do
  echo "== $D" >> gpurun_out/cfg5_phases.jsonl
  timeout -k 10 120 tools/kbench_cfg5_$D 6250000 5 >> gpurun_out/cfg5_phases.jsonl || exit 1
done
