#!/bin/bash
# Round 3: two slabs in flight for the 64-slot pass on top of stagger + priority (tools/kbench_cfg5.hip builds), then
# the full GPU suite (on 16 hardware queues via tests/conftest.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/cfg5_la64.jsonl
for rep in 1 2; do
for D in d0 la2 pr2la2; do
  echo "== $D" >> gpurun_out/cfg5_la64.jsonl
  timeout -k 10 120 tools/kbench_cfg5_$D 6250000 5 >> gpurun_out/cfg5_la64.jsonl || exit 1
done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_full2.log 2>&1
