#!/bin/bash
# Round 3: the full GPU suite (verbose, per-test timeout) with the library RR_LIBRARY names (default: in-tree).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_full.log 2>&1
