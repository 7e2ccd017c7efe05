#!/bin/bash
# SQ counter passes (8 SQ counters each) over bench --pmc-child runs of one workload (run inside gpurun).
#   bash tools/ab/sq_passes.sh gpurun_out/<dir> "<docs> <batch> <k> <dtype>"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/$1
read DOCS B K DT <<< "$2"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
W="--docs $DOCS --dtype $DT --batch $B --k $K --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --steps 3 --warmup 1"
[ -n "$EXACT" ] && W="$W --kernel exact"
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY"
P2="SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P -d "$O/p$i" -o p --output-format csv -- \
    python3 "$R/bench.py" --pmc-child --gpus 1 $W > "$O/p$i.out" 2> "$O/p$i.err" || exit 1
done
# per-kernel medians on the box; the raw per-dispatch CSVs can exceed what gpurun copies back
python3 "$R/tools/ab/sq_summary.py" "$O" > "$O/summary.json" || exit 1
[ -n "$KEEP_RAW" ] || rm -rf "$O"/p1 "$O"/p2
