# Events on launch packets: the full GPU suite, then the 125k shard with / without the exchange and the 1M headline.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu $R/tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k_$rep.json 2> $O/x125k_$rep.err &&
  timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/n125k_$rep.json 2> $O/n125k_$rep.err || exit 1
done
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/h1m.json 2> $O/h1m.err
