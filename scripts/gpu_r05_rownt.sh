#!/bin/bash
# Round 5: non-temporal gradient-row gathers (NFI_ROW_NT=1) vs plain loads — parity tests,
# then an A/B against libnfi_hip_rownt0.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_tile_check.py tests/test_gpu_deterministic.py tests/test_gpu_fullsize.py \
  > $O/rownt_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/rownt_par.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 bash scripts/ab_bench.sh $L/libnfi_hip_rownt0.so 3 --steps 20 --warmup 5 > $O/ab_rownt.log 2>&1; echo "ab rc=$?"; cat $O/ab_rownt.log
