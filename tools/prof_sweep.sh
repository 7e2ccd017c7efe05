export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 125000 250000 500000; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/sweep_$n -o run -- python3 bench.py --docs $n --steps 300 --warmup 20 --latency-steps 5 --no-cpu-baseline --no-pmc --variants "" --ingest-rows 0 > gpurun_out/sweep_$n.log 2>&1 || exit $?
done
