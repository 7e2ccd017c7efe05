# Per-call host enqueue cost at the 8-GPU shard size (tools/host_calls.py), without and with the exchange path.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/host_calls.py 125000 > $O/hostcalls.txt 2>&1 &&
timeout -k 10 120 python3 $R/tools/host_calls.py 125000 --x > $O/hostcalls_x.txt 2>&1
