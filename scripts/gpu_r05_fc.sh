#!/bin/bash
# Round 5: the fused Winograd kernel at 32 output channels per workgroup (two workgroups per CU,
# -DNFI_WINO_FC=32) against the product's 64 (one per CU): conv parity under the variant, then the
# LPIPS layer times of both builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
V=$L/libnfi_hip_DNFI_WINO_FC=32.so
timeout -k 10 300 env NFI_LIBRARY=$V python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf \
  -p no:cacheprovider tests/test_gpu_conv.py > $O/fc32_par.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 $O/fc32_par.log
[ $rc -eq 0 ] || exit 3
for r in 1 2; do
  timeout -k 10 200 python -u scripts/wino_layers.py > $O/fc64_layers_$r.log 2>&1 || exit 3
  timeout -k 10 200 env NFI_LIBRARY=$V python -u scripts/wino_layers.py > $O/fc32_layers_$r.log 2>&1 || exit 3
done
head -5 $O/fc64_layers_1.log $O/fc32_layers_1.log $O/fc64_layers_2.log $O/fc32_layers_2.log
