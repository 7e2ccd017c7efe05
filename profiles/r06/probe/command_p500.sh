# Round 6: screen phase probe (tools/gpu/r6_probe.sh), then the 500k-row shard (the default N > 1 shard: config 2 over
# a pair of ranks) through the 1-rank RCCL exchange, int8-screen chunk size 4 (default at >= 500k rows) vs 2.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6p}; mkdir -p $O; export TMPDIR=/tmp
OUT=${OUT:-r6p} bash $R/tools/gpu/r6_probe.sh || exit 1
cd /tmp
one() {
  timeout -k 10 200 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --latency-steps 50 --steady-steps 400 \
    --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --docs 500000 --exchange-1rank $2 > /tmp/ab.json 2>/tmp/ab.err || { tail -5 /tmp/ab.err; return 1; }
  python3 -c "import json; d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['steady_state']['value'], d['roofline']['screen_fallbacks_timed'])"
}
for rep in 1 2; do
  one "x500k ct4" "" >> $O/ab_500k_ct8.txt && one "x500k ct2" "--opt screen_ct8=2" >> $O/ab_500k_ct8.txt || exit 1
done
