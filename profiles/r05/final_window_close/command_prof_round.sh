#!/bin/bash
# Round profile (run inside gpurun): the driver's bench command with its PMC child pass (FETCH_SIZE, MFMA busy,
# GRBM_GUI_ACTIVE), then a rocprofv3 --kernel-trace --stats run of the same command.
#   bash tools/prof_round.sh gpurun_out/<dir>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o t --output-format csv -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --variants "" \
  > "$O/bench_traced.json" 2> "$O/trace.err" || exit 1
