#!/bin/bash
# Round 5 A/B of a tile-pass variant library (VARIANT, default ab2) against the product build: the
# parity file under the variant once, then alternating bench runs; plus the cell-run probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
V=${VARIANT:-ab2}
step() {
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
for v in $V; do
  step par_$v 240 env NFI_LIBRARY=$L/libnfi_hip_$v.so $PT tests/test_gpu_parity.py
done
[ "${PROBE:-1}" = 1 ] && step runs 200 python -u scripts/tile_runs_probe.py
for v in $V; do
  step ab_$v 500 bash scripts/ab_bench.sh $L/libnfi_hip_$v.so 3 --steps 20 --warmup 5
done
echo done
