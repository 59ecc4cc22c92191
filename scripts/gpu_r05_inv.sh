#!/bin/bash
# Round 5: kernel traces of the inversion step (vgg and l1, B=4) and the ATen op sources of the vgg step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
TAG=r05_vgg LOSS=vgg bash scripts/profile_inversion.sh || exit 3
TAG=r05_l1 LOSS=l1 bash scripts/profile_inversion.sh || exit 3
timeout -k 10 300 python -u scripts/op_sources.py vgg 4 > $O/op_sources_vgg.log 2>&1; echo "op_sources rc=$?"
tail -50 $O/op_sources_vgg.log
