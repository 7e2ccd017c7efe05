#!/bin/bash
# Round 3: hardware-queue placement of the multi-GPU data path (1-rank RCCL communicator, every block all-gathered
# and merged on the exchange lanes) at the 8-GPU shard size, and of the headline; rocprofv3 kernel traces.
set -o pipefail
mkdir -p gpurun_out/trace
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${QUEUES:-4}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace/x125k_q${QUEUES:-4} -o x125k_q${QUEUES:-4} -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" \
  --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 20 --steady-steps 40 > $GRAFT_REPO_ROOT/gpurun_out/trace/x125k_q${QUEUES:-4}.json 2> $GRAFT_REPO_ROOT/gpurun_out/trace/x125k_q${QUEUES:-4}.err
