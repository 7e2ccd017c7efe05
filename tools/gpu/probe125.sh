# Screen phase probe (tools/probe_screen) at the 8-GPU shard size: grid / chunk sweeps, and back-to-back launches.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
P=$R/tools/probe_screen
: > $O/probe125.jsonl
for args in "125000 224 2 0 1" "125000 256 2 0 1" "125000 224 1 0 1" "125000 224 4 0 1" "1000000 256 4 0 1" "125000 224 2 0 1 1"; do
  timeout -k 10 60 $P $args >> $O/probe125.jsonl 2>&1 || exit 1
done
