set -o pipefail
RR_LIBRARY=tools/ab/librag_retrieval_swz.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests13.log 2>&1 || exit 1
O=gpurun_out/ab_r13.txt
A="base:.: swz:.:RR_LIBRARY=tools/ab/librag_retrieval_swz.so"
for W in "6250000 64 10 bf16" "1000000 32 5 bf16" "1000000 32 5 fp32" "125000 32 5 fp32"; do
  bash tools/ab/ab2.sh $O "$W" $A || exit 1
done
