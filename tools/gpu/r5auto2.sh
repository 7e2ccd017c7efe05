# One query piece from 400k rows on, two in repair mode: the screen/repair GPU tests, then the driver's bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu $R/tests/test_gpu_screen.py $R/tests/test_gpu_repair.py $R/tests/test_gpu_int8.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 600 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
