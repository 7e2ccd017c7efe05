# fp32 int8 screen with one query piece (RR_SCREEN_I8_PIECES=1, the DT 9 form at 32 slots) vs two (default):
# the int8/screen/repair GPU tests under one piece, then the 1M headline and the 125k exchange path, both arms twice.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${OUT:-r5t}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
RR_SCREEN_I8_PIECES=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu -k "not proves_unit_norm" $R/tests/test_gpu_int8.py $R/tests/test_gpu_screen.py $R/tests/test_gpu_repair.py > $O/tests_p1.log 2>&1 || { tail -30 $O/tests_p1.log; exit 1; }
for rep in 1 2; do
  for P in 2 1; do
    RR_SCREEN_I8_PIECES=$P timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 --latency-steps 50 --steady-steps 500 > $O/h1m_p${P}_$rep.json 2> $O/h1m_p${P}_$rep.err || exit 1
    RR_SCREEN_I8_PIECES=$P timeout -k 10 300 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --exchange-1rank --docs 125000 --variants "" --no-cpu-baseline --no-pmc --ingest-rows 0 > $O/x125k_p${P}_$rep.json 2> $O/x125k_p${P}_$rep.err || exit 1
  done
done
# (kernel-argument placement: the screen's prologue with device-memory kernargs forced)
timeout -k 10 60 $R/tools/probe_screen 125000 224 2 0 1 > $O/probe_default.jsonl 2>&1 &&
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 $R/tools/probe_screen 125000 224 2 0 1 > $O/probe_devkernarg.jsonl 2>&1
