#!/bin/bash
# Round 3: the verify's wide phase: screen tests (ties, clustered corpora), robustness tests, clustered bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -rA \
  tests/test_gpu_screen.py tests/test_gpu_robust.py > gpurun_out/t_c.log 2>&1 &&
timeout -k 10 500 python -u tools/clustered_bench.py > gpurun_out/clustered_c.jsonl 2> gpurun_out/clustered_c.err
