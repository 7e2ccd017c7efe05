#!/bin/bash
# Round 3 final evidence, part A: full GPU suite + smoke, the driver's bench command (PMC child pass, CPU baseline) +
# rocprofv3 kernel trace and stats of the same command, SQ counter passes (headline screen, config-5 shard kernel),
# verify-kernel phase probe.
set -o pipefail
mkdir -p gpurun_out/r3g
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r3g/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3g/smoke.log 2>&1 &&
bash tools/prof_round.sh gpurun_out/r3g/driver &&
bash tools/ab/sq_passes.sh gpurun_out/r3g/sq/fp32 "1000000 32 5 fp32" &&
bash tools/ab/sq_passes.sh gpurun_out/r3g/sq/cfg5 "6250000 64 10 bf16" &&
timeout -k 10 120 tools/vprobe_bin 1000000 > gpurun_out/r3g/verify_probe.log 2>&1
