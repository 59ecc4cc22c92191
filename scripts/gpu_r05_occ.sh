#!/bin/bash
# Round 5: occupancy-4 builds of the forward (NFI_FWD_OCC=4) and the field backward (NFI_FIELD_OCC=4)
# against the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
for v in occ4 focc4; do
  timeout -k 10 400 bash scripts/ab_bench.sh $L/libnfi_hip_$v.so 2 --steps 20 --warmup 5 > $O/ab_$v.log 2>&1; echo "$v rc=$?"; cat $O/ab_$v.log
done
