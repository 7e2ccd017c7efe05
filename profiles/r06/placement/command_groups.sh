# Round 6: the exchange-thread tests after the blocking-wait change, then the bench's replica-group path on one GPU
# (two ranks as independent replicas on cuda:0: --same-device --shard-group 1), then the driver's N = 1 command.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6g}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu $R/tests/test_gpu_robust.py \
  $R/tests/test_gpu_bound_inputs.py $R/tests/test_gpu_api.py > $O/tests_x.log 2>&1 &&
timeout -k 10 300 python3 $R/bench.py --gpus 2 --same-device --shard-group 1 --no-row-shard-all --steps 20 --warmup 5 \
  --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 50 --steady-steps 200 > $O/replicas2.json 2> $O/replicas2.err &&
timeout -k 10 420 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
