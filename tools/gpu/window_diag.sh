# Why the 20-step window trails the steady state at the 125k shard: the same bench with 5, 50 and 500 warm-up steps.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for W in 5 50 500; do
  timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup $W --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 20 --steady-steps 200 > $O/n125k_w$W.json 2> $O/n125k_w$W.err || exit 1
done
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 200 --warmup 5 --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 20 --steady-steps 200 > $O/n125k_s200.json 2> $O/n125k_s200.err
