# Round-5 final evidence on the committed build: the driver's bench command with its PMC pass and the rocprofv3
# --kernel-trace --stats run of the same command (tools/prof_round.sh), then the per-GPU shard sweeps (plain and
# through the 1-rank RCCL exchange path) and the 125k exchange-path timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=gpurun_out/${OUT:-r5final}; mkdir -p $R/$O; cd /tmp; export TMPDIR=/tmp
bash $R/tools/prof_round.sh $O/prof || exit 1
bash $R/tools/shard_sweep.sh $O/shard_sweep.jsonl || exit 1
bash $R/tools/shard_sweep_x.sh $O/exchange_sweep.jsonl || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tl -o t -- python3 $R/tools/step_timeline.py run --docs 125000 --x > $R/$O/tl.out 2>&1
