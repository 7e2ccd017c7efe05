# The 8-GPU shard (125k rows) on one GPU: per-call host cost, and the bench line with and without the exchange path.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/host_calls.py 125000 --x > $O/hostcalls_x.txt 2>&1 &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k.json 2> $O/x125k.err &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/n125k.json 2> $O/n125k.err
timeout -k 10 60 $R/tools/verify_probe 125000 1 > $O/verify_probe_125k.jsonl 2>&1 &&
timeout -k 10 60 $R/tools/verify_probe 1000000 1 > $O/verify_probe_1m.jsonl 2>&1
