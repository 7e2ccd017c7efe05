# Round 6: the verify's wide phase no longer rescores the first tile's rows. The screen / int8 / bf16 / repair GPU tests
# (every wide-phase path against the exact kernel), then one vs two pieces at 125k / 250k (tools/gpu/r6_pieces.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6w}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu $R/tests/test_gpu_screen.py \
  $R/tests/test_gpu_int8.py $R/tests/test_gpu_bf16_screen.py $R/tests/test_gpu_repair.py > $O/tests_wide.log 2>&1 &&
OUT=${OUT:-r6w} bash $R/tools/gpu/r6_pieces.sh
