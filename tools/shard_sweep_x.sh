#!/bin/bash
# The multi-GPU configs' per-GPU shards on one GPU THROUGH the exchange path (bench.py --exchange-1rank: a 1-rank
# RCCL communicator, every block all-gathered on the exchange lanes and merged on the device, as each rank does).
#   bash tools/shard_sweep_x.sh gpurun_out/<file>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/$1
: > "$OUT"
while read DOCS B K DT NOTE; do
  timeout -k 10 200 python3 "$R/bench.py" --gpus 1 --exchange-1rank --docs $DOCS --batch $B --k $K --dtype $DT \
    --steps 20 --warmup 5 --latency-steps 5 --steady-steps 200 --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc \
    > /tmp/ssx.json 2>/tmp/ssx.err || { tail -3 /tmp/ssx.err >> "$OUT"; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/ssx.json').read().strip().splitlines()[-1]); s=d['steady_state']; r=d['roofline']; print(json.dumps({'workload': '$NOTE', 'docs': $DOCS, 'batch': $B, 'k': $K, 'dtype': '$DT', 'exchange': d['exchange'], 'rccl_ranks': d['rccl_ranks'], 'window_qps': d['value'], 'window_ms': d['ms_per_step'], 'steady_qps': s['value'], 'steady_ms': s['ms_per_step'], 'steady_frac': s['frac'], 'fallbacks': r.get('screen_fallbacks')}))" >> "$OUT"
done <<LIST
1000000 32 5 fp32 cfg2_1gpu_with_exchange
500000 32 5 fp32 cfg2_per_gpu_at_2
250000 32 5 fp32 cfg2_per_gpu_at_4
125000 32 5 fp32 cfg2_per_gpu_at_8
1250000 32 10 fp32 cfg3_per_gpu_at_8
6250000 64 10 bf16 cfg5_per_gpu_at_8
LIST
