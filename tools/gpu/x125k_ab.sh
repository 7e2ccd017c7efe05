# The 125k shard through the exchange path: default vs A/B arms given as environment settings, twice each.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for rep in 1 2; do
  for arm in "$@"; do
    env $arm timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k_${arm//[=,]/_}_$rep.json 2> $O/x125k_${arm//[=,]/_}_$rep.err || exit 1
  done
done
