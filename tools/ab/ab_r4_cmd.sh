set -o pipefail
O=gpurun_out/ab_r4.txt
A="s1g256:.:RR_COMPUTE_STREAMS=1 s2g224:.:RR_COMPUTE_STREAMS=2,RR_SCREEN_GRID=224 s2g208:.:RR_COMPUTE_STREAMS=2,RR_SCREEN_GRID=208"
for W in "250000 32 5 fp32" "500000 32 5 fp32" "1000000 32 10 fp32" "1250000 32 10 fp32" "2000000 32 5 fp32"; do
  bash tools/ab/ab2.sh $O "$W" $A || exit 1
done
