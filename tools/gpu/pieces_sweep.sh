# One vs two int8 query pieces across shard sizes (fp32 storage): 250k / 500k (k = 5), 1.25M / 10M (k = 10, config 3).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for W in "250000 5" "500000 5" "1250000 10" "10000000 10"; do
  read DOCS K <<< "$W"
  for P in 2 1; do
    RR_SCREEN_I8_PIECES=$P timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --docs $DOCS --k $K --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 20 --steady-steps 300 > $O/d${DOCS}_p$P.json 2> $O/d${DOCS}_p$P.err || exit 1
  done
done
