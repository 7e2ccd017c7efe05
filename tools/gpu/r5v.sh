# 32-candidate verify: screen parity tests, the 125k benches (with / without the exchange path), the verify probe.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu $R/tests/test_gpu_screen.py $R/tests/test_gpu_int8.py $R/tests/test_gpu_repair.py $R/tests/test_gpu_bf16_screen.py > $O/tests_screen.log 2>&1 ; echo "tests rc $?" >> $O/tests_screen.log
timeout -k 10 60 $R/tools/verify_probe 125000 1 > $O/verify_probe_125k.jsonl 2>&1 &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k.json 2> $O/x125k.err &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/n125k.json 2> $O/n125k.err &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/h1m.json 2> $O/h1m.err
