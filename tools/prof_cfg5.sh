#!/bin/bash
# BASELINE config-5 kernel profile on ONE MI355X (run inside gpurun): the 64-slot bf16 split-K kernel over 50M rows,
# batch 64, k 10 — the whole config-5 corpus on one device (8 GPUs hold 1/8 each).
#   bash tools/prof_cfg5.sh gpurun_out/<dir> [docs]
# 1. bench line (its own rocprofv3 --pmc child: FETCH_SIZE, SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE)
# 2. rocprofv3 --kernel-trace --stats of a short run
# 3. one SQ pass (8 SQ counters) on where the waves spend their cycles
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/$1
DOCS=${2:-50000000}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
W="--docs $DOCS --dtype bf16 --batch 64 --k 10 --no-cpu-baseline --variants= --ingest-rows 0"
timeout -k 10 400 python3 "$R/bench.py" --gpus 1 $W --steps 40 --warmup 10 --latency-steps 20 --steady-steps 40 \
  > "$O/bench.json" 2> "$O/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o t --output-format csv -- \
  python3 "$R/bench.py" --gpus 1 $W --no-pmc --steps 20 --warmup 5 --latency-steps 5 --steady-steps 5 \
  > "$O/traced.json" 2> "$O/trace.err" || exit 1
timeout -s KILL 60 rocprofv3 -L > "$O/avail.txt" 2>&1 || exit 1
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES"
for c in $SQ; do grep -q "$c" "$O/avail.txt" || { echo "missing counter $c" > "$O/sq_skipped.txt"; exit 0; }; done
timeout -s KILL 200 rocprofv3 --pmc $SQ -d "$O/sq" -o sq --output-format csv -- \
  python3 "$R/bench.py" --pmc-child --gpus 1 $W --no-pmc --steps 3 --warmup 1 \
  > "$O/sq.out" 2> "$O/sq.err" || exit 1
