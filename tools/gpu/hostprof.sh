# Host enqueue breakdown (RR_HOST_PROF=1) of the staged loop at the 8-GPU shard size, with and without the exchange path.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
RR_HOST_PROF=1 timeout -k 10 120 python3 $R/tools/step_timeline.py run --docs 125000 --x > $O/hostprof_x.txt 2>&1 &&
RR_HOST_PROF=1 timeout -k 10 120 python3 $R/tools/step_timeline.py run --docs 125000 > $O/hostprof.txt 2>&1
