#!/bin/bash
# Committed-evidence pass for one round: default bench line (N=1, with CPU baseline + PMC child pass),
# rocprofv3 kernel stats, FETCH_SIZE and MFMA counter passes of the same workload. Usage: tools/prof_round.sh TAG
TAG=${1:-r01}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 100 --warmup 10 --latency-steps 20 --no-cpu-baseline --no-pmc --variants "" --ingest-rows 0 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --latency-steps 2 --no-cpu-baseline --no-pmc --variants "" --ingest-rows 0 > gpurun_out/pmc_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -T --output-format csv -d gpurun_out/mfma_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --latency-steps 2 --no-cpu-baseline --no-pmc --variants "" --ingest-rows 0 > gpurun_out/mfma_$TAG.log 2>&1 || exit $?
for n in 125000 250000; do
  timeout -k 10 120 python bench.py --docs $n --steps 500 --no-cpu-baseline --no-pmc --variants "" --ingest-rows 0 > gpurun_out/bench_${TAG}_$n.log 2>&1 || exit $?
done
echo done
