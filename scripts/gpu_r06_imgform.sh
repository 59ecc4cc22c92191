#!/bin/bash
# Round 6: the tile pass's register-image update without the hand-written
# GPR-index regions.  Parity (parity file, full-size properties, deterministic mode) under
#   jt     -DNFI_IMG_FORM=2: wave-uniform jump table of 31 static v_add pairs (s_getpc/s_setpc)
#   native -DNFI_IMG_FORM=1: the compiler's own indexed form (img[slot] += a)
# then a 3-way A/B against the product build (ROUNDS alternating bench runs).
# (The NFI_IMG_FORM / NFI_TILE_AB / NFI_TILE_SMEM_SAFE / NFI_TILE_LDSREC knobs these libraries were
#  built with were removed once the A/B settled the form: jtd0 is the product since round 6.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
for v in jt native; do
  timeout -k 10 300 env NFI_LIBRARY=$L/libnfi_hip_$v.so python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf \
    -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_deterministic.py \
    > $O/imgform_par_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc"; tail -2 $O/imgform_par_$v.log
  [ $rc -eq 0 ] || exit 3
done
ROUNDS=3 LIBS="default $L/libnfi_hip_jt.so $L/libnfi_hip_native.so" timeout -k 10 900 bash scripts/ab_multi.sh --steps 20 --warmup 5 \
  > $O/imgform_ab.log 2>&1; echo "ab rc=$?"; cat $O/imgform_ab.log
