#!/bin/bash
# A/B of library arms x bench loops on one workload, alternating (run inside gpurun):
#   bash tools/gpu/r6_ab.sh <outdir> "<bench args>" "<arm>:<extra bench args>" ...
# arm "new" = rag-serving-system_amd/librag_retrieval.so, else tools/ab/librag_retrieval_<arm>.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
W="--no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --no-clustered --latency-steps 5 $2"
shift 2
for rep in $(seq ${REPS:-2}); do
  for spec in "$@"; do
    arm=${spec%%:*}; extra=${spec#*:}
    if [ "$arm" = new ]; then L=$R/rag-serving-system_amd/librag_retrieval.so; else L=$R/tools/ab/librag_retrieval_$arm.so; fi
    tag=$(echo "$arm $extra" | tr -c 'a-zA-Z0-9_\n' '_')
    RR_LIBRARY=$L timeout -k 10 300 python3 "$R/bench.py" --gpus 1 $W $extra > "$O/$tag.$rep.json" 2> "$O/$tag.$rep.err" || { tail -5 "$O/$tag.$rep.err"; exit 1; }
    echo "$arm [$extra] rep $rep: $(python3 $R/tools/bench_summary.py $O/$tag.$rep.json | cut -d: -f2-)" | tee -a "$O/summary.txt"
  done
done
