#!/bin/bash
# Round 3: CUs an overlapping screen leaves to the verify (RR_VERIFY_CUS 32 = default, 16, 0) at the 8-/4-GPU shards.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab_vcus.txt
REPS=3 bash tools/ab/ab2.sh gpurun_out/ab_vcus.txt "125000 32 5 fp32" v32:.:RR_VERIFY_CUS=32 v16:.:RR_VERIFY_CUS=16 v0:.:RR_VERIFY_CUS=0 &&
REPS=2 bash tools/ab/ab2.sh gpurun_out/ab_vcus.txt "250000 32 5 fp32" v32:.:RR_VERIFY_CUS=32 v16:.:RR_VERIFY_CUS=16 v0:.:RR_VERIFY_CUS=0
