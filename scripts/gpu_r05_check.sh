#!/bin/bash
# Round 5, VERDICT r04 item 1: the tile pass under the -DNFI_TILE_CHECK debug build (product layout,
# then the round-4 padded texel layout reconstructed as NFI_TEX_ROW_PAD=40, each run ONCE), then the
# product's GPU suite and an A/B bench of the grid-gradient forms.  Every step has its own time
# limit; a GPU fault (or an abort / time limit) ends the script before anything else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
step() {   # step NAME SECONDS CMD...: continue after test failures (rc 1), stop on anything worse
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 $O/$name.log
  if grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault\|HSA_STATUS_ERROR" $O/$name.log; then
    echo "GPU fault in $name: stopping"; exit 3
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit 4; fi
}
PT="python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -rf -p no:cacheprovider"
CASES="tests/test_gpu_parity.py"
step chk 240 env NFI_LIBRARY=$L/libnfi_hip_chk.so $PT $CASES
step chkpad 240 env NFI_LIBRARY=$L/libnfi_hip_chkpad.so $PT $CASES
[ "${SKIP_SUITE:-0}" = 1 ] || step suite 600 $PT tests
step ab 400 bash scripts/ab_bench.sh $L/libnfi_hip_gg0.so 2 --steps 20 --warmup 5
echo done
