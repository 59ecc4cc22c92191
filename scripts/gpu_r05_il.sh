#!/bin/bash
# Round 5: the fused Winograd kernel with the next chunk staged inside the products (NFI_WINO_INTERLEAVE=1)
# against the product: conv parity under the variant, then the LPIPS layer times of both builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
V=$L/libnfi_hip_DNFI_WINO_INTERLEAVE=1.so
timeout -k 10 300 env NFI_LIBRARY=$V python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf \
  -p no:cacheprovider tests/test_gpu_conv.py > $O/il_par.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 $O/il_par.log
[ $rc -eq 0 ] || exit 3
for r in 1 2; do
  timeout -k 10 200 python -u scripts/wino_layers.py > $O/il0_layers_$r.log 2>&1 || exit 3
  timeout -k 10 200 env NFI_LIBRARY=$V python -u scripts/wino_layers.py > $O/il_layers_$r.log 2>&1 || exit 3
done
head -5 $O/il0_layers_1.log $O/il_layers_1.log $O/il0_layers_2.log $O/il_layers_2.log
