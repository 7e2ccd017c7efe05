#!/bin/bash
# Round 3: screen epilogue rework (per-lane lists of 4 + floors, float-domain threshold): screen tests, then bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_screen.py tests/test_gpu_robust.py tests/test_gpu_api.py tests/test_gpu_configs.py > gpurun_out/t_b.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err &&
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --docs 125000 --variants "" --no-cpu-baseline --no-pmc \
  --ingest-rows 0 > gpurun_out/bench_b125k.json 2>> gpurun_out/bench_b.err
