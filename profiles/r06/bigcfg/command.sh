# Round 6: configs 3 and 5 at full size on ONE GPU (10M fp32 k = 10; 50M bf16 B = 64 k = 10), last build.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6big}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
B="--steps 20 --warmup 5 --no-cpu-baseline --variants= --ingest-rows 0 --no-pmc --no-clustered --latency-steps 20 --steady-steps 100"
timeout -k 10 400 python3 $R/bench.py --docs 10000000 --k 10 $B > $O/cfg3_10M_1gpu.json 2> $O/cfg3.err &&
timeout -k 10 500 python3 $R/bench.py --docs 50000000 --batch 64 --k 10 --dtype bf16 $B > $O/cfg5_50M_1gpu.json 2> $O/cfg5.err
