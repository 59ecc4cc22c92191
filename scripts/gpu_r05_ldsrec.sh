#!/bin/bash
# Round 5: the entry loop's records from the stage rows' pad (NFI_TILE_LDSREC=1, no scalar re-read of
# the list) — parity under the variant, then an A/B against the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 400 env NFI_LIBRARY=$L/libnfi_hip_ldsrec.so python -u -m pytest -m gpu -q --timeout 120 \
  --timeout-method thread -x -rf -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  > $O/ldsrec_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/ldsrec_par.log
grep -q "illegal memory access\|Memory access fault" $O/ldsrec_par.log && exit 3
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 bash scripts/ab_bench.sh $L/libnfi_hip_ldsrec.so 3 --steps 20 --warmup 5 > $O/ab_ldsrec.log 2>&1; echo "ab rc=$?"; cat $O/ab_ldsrec.log
