#!/bin/bash
# One parameterised GPU runner (inside gpurun): each named step writes under gpurun_out/<OUT>/ (OUT default r4),
# every GPU step under its own time limit, the steps chained so the first failure ends the call.
#   bash tools/gpu/run.sh tests smoke bench trace_x125k sq_fp32 ...
# Steps:
#   tests          the full GPU suite at the box's own GPU_MAX_HW_QUEUES (pytest -m gpu, per-test timeout)
#   tests:<file>   one test file (e.g. tests:test_gpu_screen.py)
#   smoke          __graft_entry__.smoke()
#   bench          the driver's bench command (PMC child pass, CPU baseline)
#   bench:<name>:<args>   a short bench.py run (no CPU baseline, variants, ingest or PMC pass) with extra args
#   benchenv:<name>:<VAR=value[,...]>:<args>   the same with environment settings (A/B knobs such as RR_CARRY_VERIFY=0)
#   prof           bench + rocprofv3 --kernel-trace --stats of the same command (tools/prof_round.sh)
#   trace_x125k    rocprofv3 kernel + memory-copy trace of the 1-rank RCCL exchange path at the 8-GPU shard size
#                  (Queue_Id / Stream_Id per kernel), QUEUES=4 default
#   sq_fp32 / sq_cfg5 / sq_exact   SQ counter passes (tools/ab/sq_passes.sh) on the headline / config-5 shard /
#                  exact fp32 kernel
#   sweep          per-GPU shard sweep (tools/shard_sweep.sh)
#   ab:<file>:<workload>:<arms>   A/B of library builds (tools/ab/ab.sh), e.g. "ab:ab_x.txt:1000000 32 5 fp32:x new"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r4}
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  case "$1" in
    tests) timeout -k 10 1000 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu "$R/tests" \
             > "$O/gpu_tests.log" 2>&1 ;;
    tests:*) f=${1#tests:}; timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
             "$R/tests/$f" > "$O/gpu_tests_${f%%.py*}.log" 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench) (cd /tmp && timeout -k 10 420 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" \
             2> "$O/bench.err") ;;
    bench:*) IFS=: read -r _ name bargs <<< "$1"
             (cd /tmp && timeout -k 10 300 python3 "$R/bench.py" --gpus 1 --no-cpu-baseline --variants= --ingest-rows 0 \
               --no-pmc $bargs > "$O/bench_$name.json" 2> "$O/bench_$name.err") ;;
    benchenv:*) IFS=: read -r _ name benv bargs <<< "$1"
             (cd /tmp && env $benv timeout -k 10 300 python3 "$R/bench.py" --gpus 1 --no-cpu-baseline --variants= \
               --ingest-rows 0 --no-pmc $bargs > "$O/bench_$name.json" 2> "$O/bench_$name.err") ;;
    prof) bash "$R/tools/prof_round.sh" "gpurun_out/${OUT:-r4}/prof" ;;
    trace_x125k)
      Q=${QUEUES:-4}
      mkdir -p "$O/trace_q$Q"
      (cd /tmp && GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
        -d "$O/trace_q$Q" -o x125k -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --exchange-1rank \
        --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 20 --steady-steps 40 \
        > "$O/trace_q$Q/x125k.json" 2> "$O/trace_q$Q/x125k.err") ;;
    sq_fp32) bash "$R/tools/ab/sq_passes.sh" "gpurun_out/${OUT:-r4}/sq/fp32" "1000000 32 5 fp32" ;;
    sq_cfg5) bash "$R/tools/ab/sq_passes.sh" "gpurun_out/${OUT:-r4}/sq/cfg5" "6250000 64 10 bf16" ;;
    sq_exact) EXACT=1 bash "$R/tools/ab/sq_passes.sh" "gpurun_out/${OUT:-r4}/sq/exact" "1000000 32 5 fp32" ;;
    sweep) bash "$R/tools/shard_sweep.sh" "gpurun_out/${OUT:-r4}/sweep" ;;
    ab:*) IFS=: read -r _ f w arms <<< "$1"; bash "$R/tools/ab/ab.sh" "gpurun_out/${OUT:-r4}/$f" "$w" $arms ;;
    *) echo "unknown step $1" >&2; return 2 ;;
  esac
}
for s in "$@"; do
  echo "[run.sh] $(date +%T) $s" >&2
  step "$s" || { echo "[run.sh] step $s failed (rc $?)" >&2; exit 1; }
done
