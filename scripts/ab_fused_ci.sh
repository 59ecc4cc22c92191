set -o pipefail
for r in 1 2; do
for v in 64 128; do
  NFI_FUSED_MAX_CI=$v timeout -k 10 200 python scripts/inversion_probe.py 4 vgg 30 2>&1 | grep "ms/step" | sed "s/^/ci<=$v /" || exit 1
  NFI_FUSED_MAX_CI=$v timeout -k 10 200 python scripts/inversion_probe.py 4 l1 30 2>&1 | grep "ms/step" | sed "s/^/ci<=$v /" || exit 1
done; done
