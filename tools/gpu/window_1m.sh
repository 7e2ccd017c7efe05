# Why the 1M window trails its steady state: the same bench with 5, 50 and 200 warm-up steps, and 200 timed steps.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for W in 5 50 200; do
  timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup $W --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 20 --steady-steps 300 > $O/h1m_w$W.json 2> $O/h1m_w$W.err || exit 1
done
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 200 --warmup 5 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 20 --steady-steps 300 > $O/h1m_s200.json 2> $O/h1m_s200.err
