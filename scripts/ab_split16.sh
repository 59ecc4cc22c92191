# A/B of the Winograd products (GPU box): hipBLASLt fp32 bmm vs the split-f16 GEMM, with the
# 64-channel layers on the fused kernel (FUSED_MAX_CI=64) or three-pass (0); inversion ms/step, B=4.
set -o pipefail
for r in 1 2; do
for v in "0 64" "1 64" "1 0"; do
  set -- $v
  for loss in vgg l1; do
    NFI_SPLIT16=$1 NFI_FUSED_MAX_CI=$2 timeout -k 10 200 python scripts/inversion_probe.py 4 $loss 30 2>&1 | grep "ms/step" | sed "s/^/split16=$1 ci<=$2 $loss /" || exit 1
  done
done; done
