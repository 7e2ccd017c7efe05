set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_screen.py tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests7.log 2>&1 || exit 1
O=gpurun_out/ab_r5.txt
A="new:.: cap224:.:RR_SCREEN_GRID=224 s1:.:RR_COMPUTE_STREAMS=1"
for W in "1000000 32 5 fp32" "125000 32 5 fp32"; do
  LAT=200 bash tools/ab/ab2.sh $O "$W" $A || exit 1
done
