# Round 6: the replica-group bench path with several processes on one GPU (test hook --same-device): 2 ranks as
# replicas each with a 1-rank RCCL communicator (the exchange issue thread in two processes at once), and 4 ranks as
# plain replicas. Checks the flow, not scaling (the processes share one GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6r}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
B="--steps 20 --warmup 5 --variants= --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 50 --steady-steps 200 --same-device --no-row-shard-all"
timeout -k 10 300 python3 $R/bench.py --gpus 2 --shard-group 1 --exchange-1rank $B > $O/replicas2_x.json 2> $O/replicas2_x.err &&
timeout -k 10 300 python3 $R/bench.py --gpus 4 --shard-group 1 $B > $O/replicas4.json 2> $O/replicas4.err
