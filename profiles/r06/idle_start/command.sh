# Round 6: the driver's window with the host-side batch preparation before the corpus build (default) vs after it
# (--idle-start, the GPU idle for it right before the warm-up steps); 4 alternating reps of the 1M headline.
set -o pipefail
R=$GRAFT_REPO_ROOT
REPS=4 bash $R/tools/gpu/r6_ab.sh r6idle "--steps 20 --warmup 5 --steady-steps 500" "new:" "new:--idle-start"
