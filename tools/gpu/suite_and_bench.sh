# Full GPU suite, smoke, then the headline bench and the 125k shard with and without the exchange path.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu $R/tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
(cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1) &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k.json 2> $O/x125k.err &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/n125k.json 2> $O/n125k.err &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/h1m.json 2> $O/h1m.err
