# Head-rank step of the verify's list merge with more LDS reads in flight: verify probe phases, screen tests, 125k bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5vrank}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 60 $R/tools/verify_probe 125000 1 > $O/verify_probe_125k.jsonl 2>&1 &&
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu $R/tests/test_gpu_screen.py $R/tests/test_gpu_repair.py $R/tests/test_gpu_bf16_screen.py > $O/tests.log 2>&1 &&
timeout -k 10 200 python3 $R/tools/window_cost.py 125000 --x > $O/wc_x125k.txt 2>&1 &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k.json 2> $O/x125k.err
