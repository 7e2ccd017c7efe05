# Verify phase probe (tools/verify_probe) on the int8 path at the 8-GPU shard and at 1M rows.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 60 $R/tools/verify_probe 125000 1 > $O/verify_probe_125k.jsonl 2>&1 &&
timeout -k 10 60 $R/tools/verify_probe 1000000 1 > $O/verify_probe_1m.jsonl 2>&1
