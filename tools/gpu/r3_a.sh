#!/bin/bash
# Round 3, first GPU pass: the new robustness / subnormal tests, the whole -m gpu suite, the driver's bench command,
# the clustered-corpus measurement.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_robust.py tests/test_gpu_screen.py > gpurun_out/t_new.log 2>&1 &&
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/t_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 500 python -u tools/clustered_bench.py > gpurun_out/clustered.jsonl 2> gpurun_out/clustered.err
