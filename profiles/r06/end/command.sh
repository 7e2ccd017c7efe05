# Round 6 end: the evidence for the benched HEAD.
#   bash tools/gpu/r6_final.sh suite   full GPU suite + smoke
#   bash tools/gpu/r6_final.sh prof    driver command (PMC child pass) + rocprofv3 --kernel-trace --stats of it, the SQ
#                                      passes of the screen, the per-GPU shard sweep through the 1-rank RCCL exchange
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=${OUT:-r6end}; O=$R/gpurun_out/$OUT; mkdir -p $O; export TMPDIR=/tmp
case "$1" in
  suite) OUT=$OUT bash $R/tools/gpu/run.sh tests smoke ;;
  prof) bash $R/tools/prof_round.sh gpurun_out/$OUT/prof &&
        bash $R/tools/ab/sq_passes.sh gpurun_out/$OUT/sq "1000000 32 5 fp32" &&
        bash $R/tools/shard_sweep_x.sh gpurun_out/$OUT/exchange_sweep.jsonl ;;
  *) echo "suite | prof" >&2; exit 2 ;;
esac
