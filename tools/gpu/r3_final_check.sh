#!/bin/bash
# Round 3 final check of the head: full GPU suite, smoke, and the driver's default bench command.
set -o pipefail
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r3h/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3h/smoke.log 2>&1 &&
timeout -k 10 420 python bench.py > gpurun_out/r3h/bench.json 2> gpurun_out/r3h/bench.err
