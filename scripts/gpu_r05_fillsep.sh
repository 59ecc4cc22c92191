#!/bin/bash
# Round 5: the bin fill as its own kernel (NFI_FILL_SEPARATE=1) vs the append in field_bwd: parity
# under the variant, then an A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 300 env NFI_LIBRARY=$L/libnfi_hip_fillsep.so python -u -m pytest -m gpu -q --timeout 120 \
  --timeout-method thread -x -rf -p no:cacheprovider tests/test_gpu_parity.py > $O/fillsep_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/fillsep_par.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 bash scripts/ab_bench.sh $L/libnfi_hip_fillsep.so 3 --steps 20 --warmup 5 > $O/ab_fillsep.log 2>&1; echo "ab rc=$?"; cat $O/ab_fillsep.log
