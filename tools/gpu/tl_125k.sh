# Kernel-trace timeline of the staged loop at the 8-GPU shard size without the exchange path (tools/step_timeline.py).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl0 -o t -- python3 $R/tools/step_timeline.py run --docs 125000 > $O/tl0.out 2>&1
