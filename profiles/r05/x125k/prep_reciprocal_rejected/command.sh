# Query prep by reciprocal multiply: int8 / bf16-screen / screen / repair tests, window cost and benches.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5rcp}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu $R/tests/test_gpu_int8.py $R/tests/test_gpu_bf16_screen.py $R/tests/test_gpu_screen.py $R/tests/test_gpu_repair.py > $O/tests.log 2>&1 &&
timeout -k 10 200 python3 $R/tools/window_cost.py 125000 --x > $O/wc_x125k.txt 2>&1 &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k.json 2> $O/x125k.err &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/h1m.json 2> $O/h1m.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o t --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k_traced.json 2> $O/trace.err
