#!/bin/bash
# Round 5: ATen op sources of the l1 and vgg steps, and the l1 step's kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python -u scripts/op_sources.py l1 4 > $O/op_sources_l1.log 2>&1; echo "l1 rc=$?"
timeout -k 10 300 python -u scripts/op_sources.py vgg 4 > $O/op_sources_vgg2.log 2>&1; echo "vgg rc=$?"
TAG=r05_l1b LOSS=l1 bash scripts/profile_inversion.sh || exit 3
TAG=r05_vggb LOSS=vgg bash scripts/profile_inversion.sh || exit 3
