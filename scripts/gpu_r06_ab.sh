#!/bin/bash
# Round 6: A/B of the in-tree product against variant libraries (LIBS, space-separated names under
# nfi/: libnfi_hip_NAME.so), ROUNDS alternating bench runs, renderer only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
LIBS_FULL="default"
for v in ${VARIANTS}; do LIBS_FULL="$LIBS_FULL $L/libnfi_hip_$v.so"; done
ROUNDS=${ROUNDS:-3} LIBS="$LIBS_FULL" timeout -k 10 900 bash scripts/ab_multi.sh --steps 20 --warmup 5 \
  > $O/ab_${TAG:-x}.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/ab_${TAG:-x}.log; exit $rc
