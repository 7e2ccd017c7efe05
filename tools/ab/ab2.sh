#!/bin/bash
# A/B of bench arms interleaved on one GPU box (run inside gpurun). An arm is name:dir:ENV=VAL[,ENV=VAL]
# (dir holds the bench.py + package to run; "." = the working tree). Arms alternate REPS times per workload.
# (r6: the product library reads path options through rr_set_option only — set them with EXTRA="--opt name=value",
# or give an arm a library built with tools/ab/build_rev.sh ... -DRR_AB_ENV=1, which reads RR_<NAME> variables.)
#   bash tools/ab/ab2.sh gpurun_out/<file> "<docs> <batch> <k> <dtype>" arm1 arm2 ...
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/$1
read DOCS B K DT <<< "$2"
shift 2
W="${EXTRA:-} --docs $DOCS --dtype $DT --batch $B --k $K --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --steps ${STEPS:-20} --warmup ${WARMUP:-5} --latency-steps ${LAT:-5} --steady-steps ${STEADY:-200}"
echo "# $DOCS rows, batch $B, k $K, $DT: window value ms kernel_us | steady value ms kernel_us" >> "$OUT"
for rep in $(seq ${REPS:-2}); do
  for arm in "$@"; do
    IFS=: read NAME DIR ENVS <<< "$arm"
    ( cd "$R/$DIR" && env ${ENVS//,/ } timeout -k 10 200 python3 bench.py --gpus 1 $W > /tmp/ab.json 2>/tmp/ab.err ) || { echo "$NAME FAILED" >> "$OUT"; tail -5 /tmp/ab.err >> "$OUT"; exit 1; }
    python3 -c "import json; d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]); s=d['steady_state']; r=d['roofline']; print('$NAME', d['value'], d['ms_per_step'], r['kernel_avg_us'], '| steady', s['value'], s['ms_per_step'], s['kernel_avg_us'], '| p50/p99', d['p50_ms'], d['p99_ms'], '| pipe', d['host_pipelined']['value'], '| fb', r.get('screen_fallbacks'), '/', r.get('screened_blocks'))" >> "$OUT"
  done
done
