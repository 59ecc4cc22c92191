#!/bin/bash
# Round 5: the augmented copies' adjoint re-mapped (one copy per wave, coalesced): its parity tests,
# the vgg inversion step's kernel trace, and the step's generic GEMM shapes.
set -u
PATTERNS="13" bash scripts/gpu_r05_idx8.sh || exit 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_lpips.py > $O/aug_par.log 2>&1
rc=$?; echo "lpips tests rc=$rc"; tail -2 $O/aug_par.log
[ $rc -eq 0 ] || exit 3
TAG=r05_aug LOSS=vgg STEPS=8 bash scripts/profile_inversion.sh || exit 3
timeout -k 10 300 python -u scripts/gemm_shapes_probe.py vgg 4 > $O/gemm_shapes_vgg.log 2>&1; echo "shapes rc=$?"
head -20 $O/gemm_shapes_vgg.log
