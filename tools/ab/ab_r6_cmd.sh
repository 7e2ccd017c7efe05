set -o pipefail
O=gpurun_out/ab_r6.txt
A="new:.: nochain:.:RR_X_NOCHAIN=1 norec:.:RR_X_NOCHAIN=1,RR_X_NOREC=1"
for W in "125000 32 5 fp32" "1000000 32 5 fp32"; do
  STEPS=200 WARMUP=20 bash tools/ab/ab2.sh $O "$W" $A || exit 1
done
