# Round 6: staging followed by a wait-value packet (option stage_wait_value) on a staging stream vs the default (the
# next block's compute stream); alternating arms, 125k through the 1-rank RCCL exchange and 1M. Lines: arm, window q/s,
# steady q/s.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6s}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
one() {   # name, workload args, options
  timeout -k 10 200 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --latency-steps 50 --steady-steps 400 \
    --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc $2 $3 > /tmp/ab.json 2>/tmp/ab.err || { tail -5 /tmp/ab.err; return 1; }
  python3 -c "import json; d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['steady_state']['value'], d['roofline']['screen_fallbacks_timed'])"
}
for W in "x125k:--docs 125000 --exchange-1rank" "1M:--docs 1000000"; do
  n=${W%%:*}; a=${W#*:}
  for rep in 1 2; do
    one "$n default" "$a" "" >> $O/stage_ab.txt &&
    one "$n s1_wv1" "$a" "--opt stage_stream=1 --opt stage_wait_value=1" >> $O/stage_ab.txt &&
    one "$n s2_wv1" "$a" "--opt stage_stream=2 --opt stage_wait_value=1" >> $O/stage_ab.txt &&
    one "$n s1_wv0" "$a" "--opt stage_stream=1" >> $O/stage_ab.txt || exit 1
  done
done
