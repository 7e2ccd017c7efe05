# One query piece from 400k rows on: the full GPU suite, smoke, then the driver's bench command (clustered field,
# variants, PMC pass, CPU baseline).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu $R/tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
(cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1) &&
timeout -k 10 600 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
