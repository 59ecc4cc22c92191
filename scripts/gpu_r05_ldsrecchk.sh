#!/bin/bash
# Round 5: the LDS-record variant's failing parity case under the integrity-check build (code 6 now
# also compares the entry loop's LDS records with the batch's vector records).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 300 env NFI_LIBRARY=$L/libnfi_hip_ldsrecchk.so python -u -m pytest -m gpu -q --timeout 120 \
  --timeout-method thread -rf -p no:cacheprovider tests/test_gpu_parity.py -k "field_heads_seeded or binning" \
  > $O/ldsrecchk.log 2>&1
echo "rc=$?"; grep -E "passed|failed|tile check|AssertionError|NfiError" $O/ldsrecchk.log | head -12
