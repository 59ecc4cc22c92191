#!/bin/bash
# Round 5: cell sub-bins (NFI_CELL_BINS) — parity and check-build tests, the cell-run probe, then an
# A/B against the tile-bin build (libnfi_hip_tilebins.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault\|HSA_STATUS_ERROR" "$1"; }
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_tile_check.py tests/test_gpu_torch_ops.py > $O/cells_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -5 $O/cells_par.log
fault $O/cells_par.log && exit 3
[ $rc -eq 0 ] || exit 3
timeout -k 10 200 python -u scripts/tile_runs_probe.py > $O/cells_runs.log 2>&1; echo "runs rc=$?"; tail -6 $O/cells_runs.log
timeout -k 10 600 bash scripts/ab_bench.sh $L/libnfi_hip_tilebins.so 3 --steps 20 --warmup 5 > $O/ab_cells.log 2>&1; echo "ab rc=$?"; cat $O/ab_cells.log
timeout -k 10 200 python -u scripts/stamps.py > $O/stamps_cells.log 2>&1; echo "stamps rc=$?"; tail -28 $O/stamps_cells.log
