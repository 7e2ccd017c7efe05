#!/bin/bash
# Round 3: static issue priority for one half of the SIMD partners (tools/kbench_cfg5.hip builds), config-5 shard.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/cfg5_prio.jsonl
for rep in 1 2; do
for D in d0 p1 p2 p1s0; do
  echo "== $D" >> gpurun_out/cfg5_prio.jsonl
  timeout -k 10 120 tools/kbench_cfg5_$D 6250000 5 >> gpurun_out/cfg5_prio.jsonl || exit 1
done
done
