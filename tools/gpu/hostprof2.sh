# Host-side costs: HIP call microbenchmark and the exchange path's per-call host profile (RR_HOST_PROF=1).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 60 $R/tools/api_cost > $O/api_cost.json 2>&1 &&
RR_HOST_PROF=1 timeout -k 10 120 python3 $R/tools/host_calls.py 125000 --x > $O/hostprof_x2.txt 2>&1
