# Round 6: one vs two int8 query pieces on the small shards (125k, 250k) through the 1-rank RCCL exchange, on the r6
# build (staged pieces, host geometry); 2 alternating reps. Lines: arm, window q/s, steady q/s, flagged, wide-phase slots.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6q}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
one() {
  timeout -k 10 200 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --latency-steps 50 --steady-steps 400 \
    --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --exchange-1rank $2 > /tmp/ab.json 2>/tmp/ab.err || { tail -5 /tmp/ab.err; return 1; }
  python3 -c "import json; d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', d['value'], d['steady_state']['value'], r['screen_fallbacks_timed'], r['wide_verified_slots_timed'])"
}
for D in 125000 250000; do
  for rep in 1 2; do
    one "$D p2" "--docs $D" >> $O/ab_pieces.txt && one "$D p1" "--docs $D --opt screen_i8_pieces=1" >> $O/ab_pieces.txt || exit 1
  done
done
