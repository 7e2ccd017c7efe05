# Round 6: config 4 (SQuAD end to end: e5-large-shaped random-weight encoder + HIP retriever) and the serving-level
# replay of the reference's load-test traces (retrieval-only table encoder, and the e5-shaped encoder), last build.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r6srv}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 python3 $R/tools/bench_e2e.py > $O/bench_cfg4_squad_e2e_1gpu.jsonl 2> $O/e2e.err &&
timeout -k 10 400 python3 $R/tools/serve_replay.py --encoder table > $O/serve_table.jsonl 2> $O/serve_table.err &&
timeout -k 10 400 python3 $R/tools/serve_replay.py --encoder e5 --rps 50,200,1000 > $O/serve_e5.jsonl 2> $O/serve_e5.err
