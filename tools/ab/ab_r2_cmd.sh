set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_screen.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests3.log 2>&1 || exit 1
O=gpurun_out/ab_r2.txt
A="s1:.:RR_COMPUTE_STREAMS=1 s2:.:RR_COMPUTE_STREAMS=2 s1o:.:RR_COMPUTE_STREAMS=1,RR_LIBRARY=tools/ab/librag_retrieval_onep.so s2o:.:RR_COMPUTE_STREAMS=2,RR_LIBRARY=tools/ab/librag_retrieval_onep.so"
for W in "125000 32 5 fp32" "250000 32 5 fp32" "500000 32 5 fp32" "1000000 32 5 fp32" "1250000 32 10 fp32" "1000000 32 10 fp32"; do
  bash tools/ab/ab2.sh $O "$W" $A || exit 1
done
