# Marker/barrier device costs (tools/api_cost), the multi-process GPU tests, and the 125k shard through the exchange path.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 90 $R/tools/api_cost > $O/api_cost5.json 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu -k "dist or rccl or rank or exchange or async or shards or stage or stream" $R/tests > $O/tests_x.log 2>&1 || { tail -30 $O/tests_x.log; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k_$rep.json 2> $O/x125k_$rep.err || exit 1
done
timeout -k 10 120 python3 $R/tools/host_calls.py 125000 --x > $O/hostcalls_x.txt 2>&1
