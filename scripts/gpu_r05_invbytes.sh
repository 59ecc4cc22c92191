#!/bin/bash
# Round 5: HBM bytes per kernel of the inversion step (FETCH_SIZE and WRITE_SIZE, separate passes) and
# its kernel trace, to find kernels whose traffic exceeds their algorithmic bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/invbytes; mkdir -p $OUT
CMD="scripts/inversion_probe.py 4 ${LOSS:-vgg} 6"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $CMD > $OUT/trace.log 2>&1 || exit 3
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 $CMD > $OUT/$c.log 2>&1 || exit 3
done
find $OUT/trace -name "*kernel_trace.csv" -delete
echo done
