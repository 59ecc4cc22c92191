#!/bin/bash
# Round 5: the tile pass with no scalar record load in flight across an indexed region
# (-DNFI_TILE_SMEM_SAFE=1): parity under the variant, then an A/B against the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
V=$L/libnfi_hip_smemsafe.so
timeout -k 10 400 env NFI_LIBRARY=$V python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf \
  -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_deterministic.py \
  > $O/smemsafe_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/smemsafe_par.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 bash scripts/ab_bench.sh $V 3 --steps 20 --warmup 5 > $O/ab_smemsafe.log 2>&1; echo "ab rc=$?"; cat $O/ab_smemsafe.log
