#!/bin/bash
# SQ counter pass (one pass, <= 8 SQ counters) of the screen over library arms (run inside gpurun):
#   bash tools/gpu/r6_sq.sh <outdir> "<bench args>" "<counters>" arm ...
# arm "new" = rag-serving-system_amd/librag_retrieval.so, else tools/ab/librag_retrieval_<arm>.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
W="--gpus 1 --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --no-clustered --steps 3 --warmup 1 --latency-steps 2 --steady-steps 5 $2"
C=$3
shift 3
cd /tmp && export TMPDIR=/tmp
for arm in "$@"; do
  if [ "$arm" = new ]; then L=$R/rag-serving-system_amd/librag_retrieval.so; else L=$R/tools/ab/librag_retrieval_$arm.so; fi
  RR_LIBRARY=$L timeout -s KILL 200 rocprofv3 --pmc $C -d "$O/$arm" -o p --output-format csv -- \
    python3 "$R/bench.py" --pmc-child $W > "$O/$arm.out" 2> "$O/$arm.err" || { tail -5 "$O/$arm.err"; exit 1; }
  python3 "$R/tools/ab/sq_summary.py" "$O/$arm" > "$O/$arm.summary.json" || exit 1
  rm -rf "$O/$arm"
done
