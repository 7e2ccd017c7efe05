# 50M bf16 rows on one GPU (B = 64, k = 10): repair mode / full lists from the start (option screen_full_lists) vs default.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6fl}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
B="--docs 50000000 --batch 64 --k 10 --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --no-clustered --latency-steps 20 --steady-steps 100"
timeout -k 10 500 python3 $R/bench.py $B --opt screen_full_lists=1 > $O/cfg5_50M_fl.json 2> $O/fl.err &&
timeout -k 10 500 python3 $R/bench.py $B > $O/cfg5_50M_default.json 2> $O/def.err
