set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5t; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o t -- python3 $R/tools/step_timeline.py run --docs 125000 --x > $O/tl.out 2>&1 &&
timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k.json 2> $O/x125k.err
