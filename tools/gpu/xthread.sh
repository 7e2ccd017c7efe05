# Exchange issue thread: the multi-process (1-rank RCCL) GPU tests, then the 125k shard through the exchange path with
# the thread (default) and without it (RR_X_THREAD=0), twice each, and the per-call host cost.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu -k "dist or rccl or rank or exchange or async or shards" $R/tests > $O/tests_x.log 2>&1 || { tail -30 $O/tests_x.log; exit 1; }
for rep in 1 2; do
  for T in 1 0; do
    RR_X_THREAD=$T timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k_t${T}_$rep.json 2> $O/x125k_t${T}_$rep.err || exit 1
  done
done
timeout -k 10 120 python3 $R/tools/host_calls.py 125000 --x > $O/hostcalls_x.txt 2>&1
