#!/bin/bash
# Round 5 closing run: the GPU suite and the default bench on the final tree, then the kernel traces
# of both inversion steps (scripts/inversion_step_table.py summarises them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05_v5}
SKIP_PROF=1 TAG=$TAG bash scripts/gpu_r05_round.sh || exit 3
TAG=${TAG}_vgg LOSS=vgg STEPS=8 bash scripts/profile_inversion.sh || exit 3
TAG=${TAG}_l1 LOSS=l1 STEPS=8 bash scripts/profile_inversion.sh || exit 3
echo done
