#!/bin/bash
# Round 6, second call: the jump-table image update (no GPR-index mode) lets scalar record loads stay
# in flight across the entry loop (jt0 = NFI_TILE_SMEM_SAFE=0, the round-5 fast schedule) or the
# records come from the stage rows (jtl = NFI_TILE_LDSREC=1).  Parity under each; the variants that
# pass go into an A/B against the product and jt (ROUNDS alternating bench runs).
# (The NFI_IMG_FORM / NFI_TILE_AB / NFI_TILE_SMEM_SAFE / NFI_TILE_LDSREC knobs these libraries were
#  built with were removed once the A/B settled the form: jtd0 is the product since round 6.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
LIBS="default"
for v in ${VARIANTS:-jt0 jtl}; do
  timeout -k 10 300 env NFI_LIBRARY=$L/libnfi_hip_$v.so python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf \
    -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_deterministic.py \
    > $O/imgform2_par_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc"; tail -2 $O/imgform2_par_$v.log
  [ $rc -eq 0 ] && LIBS="$LIBS $L/libnfi_hip_$v.so"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3    # (a crash / timeout ends the call)
done
ROUNDS=3 LIBS="$LIBS" timeout -k 10 900 bash scripts/ab_multi.sh --steps 20 --warmup 5 \
  > $O/imgform2_ab.log 2>&1; echo "ab rc=$?"; cat $O/imgform2_ab.log
