#!/bin/bash
# Round 5: the augmented-copy adjoint's box walk four columns per pass: its tests and the vgg step trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_lpips.py > $O/aug2_par.log 2>&1
rc=$?; echo "lpips tests rc=$rc"; tail -2 $O/aug2_par.log
[ $rc -eq 0 ] || exit 3
TAG=r05_aug2 LOSS=vgg STEPS=8 bash scripts/profile_inversion.sh || exit 3
grep aug_ gpurun_out/prof_inv_r05_aug2/trace/run_kernel_stats.csv | cut -c1-160
