#!/bin/bash
# Round 3 final: the screened search on clustered SQuAD-derived 1M corpora vs the exact kernel (tools/clustered_bench.py).
set -o pipefail
mkdir -p gpurun_out/r3h
timeout -k 10 900 python -u tools/clustered_bench.py > gpurun_out/r3h/clustered.jsonl 2> gpurun_out/r3h/clustered.err
