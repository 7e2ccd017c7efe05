# Exchange-path diagnosis at the 125k shard: per-call host cost (with and without the exchange) and a kernel-trace
# timeline of the staged loop with the exchange.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/host_calls.py 125000 --x > $O/hostcalls_x.txt 2>&1 &&
timeout -k 10 120 python3 $R/tools/host_calls.py 125000 > $O/hostcalls.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o t -- python3 $R/tools/step_timeline.py run --docs 125000 --x > $O/tl.out 2>&1
