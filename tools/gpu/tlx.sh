# Kernel-trace timeline of the staged loop through the exchange path (tools/step_timeline.py --x).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o t -- python3 $R/tools/step_timeline.py run --docs 125000 --x > $O/tl.out 2>&1
