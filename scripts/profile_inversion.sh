#!/bin/bash
# rocprofv3 kernel trace of the inversion step (B images, loss, steps): which kernels own s/image.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_inv_${TAG:-r01}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 scripts/inversion_probe.py ${B:-4} ${LOSS:-vgg} ${STEPS:-10} > $OUT/trace.log 2>&1 || exit $?
tail -2 $OUT/trace.log
