#!/bin/bash
# One GPU session: smoke -> gpu tests -> bench -> rocprofv3 kernel stats -> PMC (FETCH_SIZE) pass.
# Stops at the first crash/timeout (exit > 1). Usage: tools/gpu_check.sh [tag] [pytest-marker-expr]
TAG=${1:-r01}
cd "$(dirname "$0")/.."
MARK=${2:-"gpu and not big"}
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1200 python -m pytest tests -q -m "$MARK" --timeout 600 -p no:cacheprovider
step bench 600 python bench.py
step prof_stats 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 100 --warmup 10 --latency-steps 20 --no-cpu-baseline --no-pmc --variants "" --ingest-rows 0
step prof_pmc 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --latency-steps 2 --no-cpu-baseline --no-pmc --variants "" --ingest-rows 0
step prof_mfma 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -T --output-format csv -d gpurun_out/mfma_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --latency-steps 2 --no-cpu-baseline --no-pmc --variants "" --ingest-rows 0
