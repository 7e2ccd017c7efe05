# Round 6: kernel units loaded at rr_create (preload_kernels). API + parity GPU tests, then the driver's command and its
# rocprofv3 trace (tools/prof_round.sh): the first search without the deferred-load stall.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=${OUT:-r6pl}; O=$R/gpurun_out/$OUT; mkdir -p $O; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu $R/tests/test_gpu_api.py \
  $R/tests/test_gpu_parity.py > $O/tests.log 2>&1) && bash $R/tools/prof_round.sh gpurun_out/$OUT/prof
