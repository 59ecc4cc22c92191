#!/bin/bash
# Round 5: A/B of the in-tree build against libnfi_hip_prev.so (the build before the change), with
# the parity file first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_parity.py > $O/abprev_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/abprev_par.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 bash scripts/ab_bench.sh $L/libnfi_hip_prev.so 3 --steps 20 --warmup 5 > $O/abprev.log 2>&1; echo "ab rc=$?"; cat $O/abprev.log
