#!/bin/bash
# Round-6 GPU step: selected GPU tests, then the bench in the given dtypes (each step time-limited, chained).
#   bash tools/gpu/r6_step.sh <outdir> "<pytest files>" "<bench dtypes>" [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
cd "$R" || exit 1
if [ -n "$2" ]; then
  timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread $2 > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
  tail -3 "$O/tests.log"
fi
for dt in $3; do
  timeout -k 10 400 python3 bench.py --dtype $dt --no-cpu-baseline --no-pmc --no-clustered --ingest-rows 0 $4 > "$O/bench_$dt.json" 2> "$O/bench_$dt.err" || { tail -20 "$O/bench_$dt.err"; exit 1; }
  python3 tools/bench_summary.py "$O/bench_$dt.json" 2>/dev/null || tail -c 600 "$O/bench_$dt.json"
done
