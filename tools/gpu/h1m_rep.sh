# The 1M headline's 20-step window, five times on one box (window variance), short form.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for rep in 1 2 3 4 5; do
  timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 50 --steady-steps 500 > $O/h1m_$rep.json 2> $O/h1m_$rep.err || exit 1
done
