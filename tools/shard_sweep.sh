#!/bin/bash
# Per-GPU shard sizes of the multi-GPU configs, measured on one GPU (run inside gpurun): the driver window
# (--steps 20 --warmup 5) and the steady state, one line per workload.
#   bash tools/shard_sweep.sh gpurun_out/<file>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/$1
: > "$OUT"
while read DOCS B K DT NOTE; do
  timeout -k 10 200 python3 "$R/bench.py" --gpus 1 --docs $DOCS --batch $B --k $K --dtype $DT --steps 20 --warmup 5 \
    --latency-steps 5 --steady-steps 200 --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc > /tmp/ss.json 2>/tmp/ss.err \
    || { tail -3 /tmp/ss.err >> "$OUT"; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/ss.json').read().strip().splitlines()[-1]); s=d['steady_state']; r=d['roofline']; print(json.dumps({'workload': '$NOTE', 'docs': $DOCS, 'batch': $B, 'k': $K, 'dtype': '$DT', 'window_qps': d['value'], 'window_ms': d['ms_per_step'], 'window_kernel_us': r['kernel_avg_us'], 'steady_qps': s['value'], 'steady_ms': s['ms_per_step'], 'steady_kernel_us': s['kernel_avg_us'], 'steady_frac': s['frac'], 'alg_bytes': r['alg_bytes_per_launch'], 'fallbacks': r.get('screen_fallbacks'), 'host_enqueue_ms': d.get('host_enqueue_ms_per_step')}))" >> "$OUT"
done <<LIST
1000000 32 5 fp32 cfg2_1gpu
500000 32 5 fp32 cfg2_per_gpu_at_2
250000 32 5 fp32 cfg2_per_gpu_at_4
125000 32 5 fp32 cfg2_per_gpu_at_8
10000000 32 10 fp32 cfg3_on_1gpu
1250000 32 10 fp32 cfg3_per_gpu_at_8
50000000 64 10 bf16 cfg5_on_1gpu
6250000 64 10 bf16 cfg5_per_gpu_at_8
1000000 32 5 bf16 cfg2_bf16
LIST
