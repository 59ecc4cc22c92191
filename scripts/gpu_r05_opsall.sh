#!/bin/bash
# Round 5: device time of every ATen op of the vgg and l1 inversion steps by input shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u scripts/gemm_shapes_probe.py vgg 4 all > $O/ops_all_vgg.log 2>&1; echo "vgg rc=$?"
timeout -k 10 300 python -u scripts/gemm_shapes_probe.py l1 4 all > $O/ops_all_l1.log 2>&1; echo "l1 rc=$?"
grep "ms/step" $O/ops_all_vgg.log | head -45
