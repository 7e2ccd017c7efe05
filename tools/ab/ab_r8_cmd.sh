set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests9.log 2>&1 || exit 1
O=gpurun_out/ab_r8.txt
for D in 0 30 50; do
  echo "## exchange delay $D us (1-rank RCCL exchange), two exchange lanes" >> $O
  A="x4l2:.:RR_X_EXCHANGE_DELAY_US=$D"
  EXTRA=--exchange-1rank bash tools/ab/ab2.sh $O "125000 32 5 fp32" $A || exit 1
done
EXTRA=--exchange-1rank bash tools/ab/ab2.sh $O "1000000 32 5 fp32" x4l2:.: || exit 1
