#!/bin/bash
# Round 3: adaptive screen (short -> full lane lists -> pause): screen tests, clustered bench, headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -rA \
  tests/test_gpu_screen.py > gpurun_out/t_d.log 2>&1 &&
timeout -k 10 600 python -u tools/clustered_bench.py > gpurun_out/clustered_d.jsonl 2> gpurun_out/clustered_d.err &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --variants "" --no-cpu-baseline --no-pmc \
  --ingest-rows 0 > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err
