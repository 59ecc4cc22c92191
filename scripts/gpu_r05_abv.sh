#!/bin/bash
# Round 5: one entry-form variant library (AB=$V) through the parity tests, once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 240 env NFI_LIBRARY=$L/libnfi_hip_$V.so python -u -m pytest -m gpu -q --timeout 120 \
  --timeout-method thread -x -rf -p no:cacheprovider tests/test_gpu_parity.py > $O/par_$V.log 2>&1
rc=$?; echo "par_$V rc=$rc"; grep -E "passed|failed|Error" $O/par_$V.log | head -8
exit 0
