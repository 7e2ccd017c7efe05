set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests8.log 2>&1 || exit 1
O=gpurun_out/ab_r7.txt
for D in 0 30; do
  echo "## exchange delay $D us (1-rank RCCL exchange)" >> $O
  A="x4:.:RR_X_EXCHANGE_DELAY_US=$D x2:.:RR_X_SLOTS=2,RR_X_EXCHANGE_DELAY_US=$D"
  EXTRA=--exchange-1rank bash tools/ab/ab2.sh $O "125000 32 5 fp32" $A || exit 1
done
