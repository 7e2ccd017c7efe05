#!/bin/bash
# Round 3 A/B: GPU_MAX_HW_QUEUES 4 vs 16 on the multi-GPU data path (1-rank RCCL, 125k rows) and the headline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/ab_queues.txt
rm -f $OUT
W="--gpus 1 --steps 20 --warmup 5 --variants= --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 50 --steady-steps 100"
for rep in 1 2; do
  for q in 4 16; do
    for cfg in "--exchange-1rank --docs 125000" "--docs 1000000"; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py $W $cfg > /tmp/q.json 2> /tmp/q.err || { tail -3 /tmp/q.err >> $OUT; exit 1; }
      python3 -c "import json; d=json.loads(open('/tmp/q.json').read().strip().splitlines()[-1]); print('queues $q', '$cfg', d['value'], '| steady', d['steady_state']['value'], '| p50', d['p50_ms'], '| pipelined', d['host_pipelined']['value'])" >> $OUT
    done
  done
done
