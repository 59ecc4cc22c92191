#!/bin/bash
# Round 5: per-phase stamps of the product and the early bin-append variant, an A/B of the two,
# then (last: it may fault) the AB=6 entry-form experiment's parity run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault\|HSA_STATUS_ERROR" "$1"; }
timeout -k 10 200 python -u scripts/stamps.py > $O/stamps_prod.log 2>&1; rc=$?; echo "stamps rc=$rc"; cat $O/stamps_prod.log | tail -28
[ $rc -eq 0 ] || exit 3
NFI_STAMPS_LIB=$L/libnfi_hip_stamps_early.so timeout -k 10 200 python -u scripts/stamps.py > $O/stamps_early.log 2>&1; rc=$?; echo "stamps early rc=$rc"; tail -12 $O/stamps_early.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 bash scripts/ab_bench.sh $L/libnfi_hip_early.so 3 --steps 20 --warmup 5 > $O/ab_early.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/ab_early.log
[ $rc -eq 0 ] || exit 3
if [ "${AB6:-1}" = 1 ]; then
  timeout -k 10 240 env NFI_LIBRARY=$L/libnfi_hip_ab6.so python -u -m pytest -m gpu -q --timeout 120 \
    --timeout-method thread -x -rf -p no:cacheprovider tests/test_gpu_parity.py > $O/par_ab6.log 2>&1
  echo "par_ab6 rc=$?"; grep -E "passed|failed|Error" $O/par_ab6.log | head -5
fi
exit 0
