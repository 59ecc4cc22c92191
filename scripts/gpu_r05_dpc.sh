#!/bin/bash
# Round 5: plane-major grid-gradient buffer (NFI_DPC_PLANAR=1) vs [sample][plane] — parity tests,
# then an A/B against libnfi_hip_dpc0.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_tile_check.py tests/test_gpu_deterministic.py tests/test_gpu_fullsize.py \
  > $O/dpc_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/dpc_par.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 bash scripts/ab_bench.sh $L/libnfi_hip_dpc0.so 3 --steps 20 --warmup 5 > $O/ab_dpc.log 2>&1; echo "ab rc=$?"; cat $O/ab_dpc.log
