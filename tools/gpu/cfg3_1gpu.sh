# Config 3's corpus on one GPU (10M rows, k = 10) on the current build (one query piece capped below 4M rows).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --gpus 1 --docs 10000000 --k 10 --steps 20 --warmup 5 --latency-steps 5 --steady-steps 200 --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc > $O/cfg3_1gpu.json 2> $O/cfg3_1gpu.err
