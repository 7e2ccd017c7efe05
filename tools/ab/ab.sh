#!/bin/bash
# A/B of library builds on one workload, arms alternating twice (run inside gpurun).
#   bash tools/ab/ab.sh gpurun_out/<file> "<docs> <batch> <k> <dtype>" arm1 arm2 ...
# arm "new" = rag-serving-system_amd/librag_retrieval.so, else tools/ab/librag_retrieval_<arm>.so
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/$1
read DOCS B K DT <<< "$2"
shift 2
W="--docs $DOCS --dtype $DT --batch $B --k $K --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --steps ${STEPS:-40} --warmup ${WARMUP:-10} --latency-steps 5 --steady-steps 60 $EXTRA"
echo "# $DOCS rows, batch $B, k $K, $DT: value kernel_us frac | steady value kernel_us frac" >> "$OUT"
for rep in $(seq ${REPS:-2}); do
  for arm in "$@"; do
    if [ $arm = new ]; then L=$R/rag-serving-system_amd/librag_retrieval.so; else L=$R/tools/ab/librag_retrieval_$arm.so; fi
    RR_LIBRARY=$L timeout -k 10 200 python3 "$R/bench.py" --gpus 1 $W > /tmp/ab.json 2>/tmp/ab.err || { tail -5 /tmp/ab.err >> "$OUT"; exit 1; }
    python3 -c "import json; d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]); s=d['steady_state']; print('$arm', d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], 'alone', (d['roofline'].get('kernel_alone') or {}).get('kernel_avg_us'), '| steady', s['value'], s['kernel_avg_us'], s['frac'], '| fallbacks', d['roofline'].get('screen_fallbacks'), '/', d['roofline'].get('screened_blocks'))" >> "$OUT"
  done
done
