#!/bin/bash
# Round 5: ray-striped sub-bins (NFI_KEY_STRIPES, product 8) — parity + check-build tests under the
# product, then an A/B against the unstriped build (libnfi_hip_stripes1.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_tile_check.py tests/test_gpu_torch_ops.py > $O/stripes_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/stripes_par.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 bash scripts/ab_bench.sh $L/libnfi_hip_stripes1.so 3 --steps 20 --warmup 5 > $O/ab_stripes.log 2>&1; echo "ab rc=$?"; cat $O/ab_stripes.log
