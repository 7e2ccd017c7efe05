# Round 6: the staging kernel's sums by DPP. The int8 / bf16-screen / bound-input GPU tests (the staged scalars feed every
# int8 bound), the staging kernel alone, then 125k through the exchange (the staging sits on each compute stream's
# chain there) and the 1M headline, 2 reps each against the previous build (arm predpp).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6d}; mkdir -p $O; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu $R/tests/test_gpu_int8.py \
  $R/tests/test_gpu_bf16_screen.py $R/tests/test_gpu_bound_inputs.py $R/tests/test_gpu_screen.py > $O/tests.log 2>&1) &&
OUT=${OUT:-r6d} bash $R/tools/gpu/r6_stage_alone.sh &&
REPS=2 bash $R/tools/gpu/r6_ab.sh ${OUT:-r6d}/x125k "--steps 20 --warmup 5 --steady-steps 1000 --docs 125000 --exchange-1rank" "predpp:" "new:"
