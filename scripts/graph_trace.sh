#!/bin/bash
# why does the HIP-graph replay of the inversion step run the GPU slower than
# the eager loop?  Kernel traces of bench.py's inversion leg (B = 4, LOSS, 10 steps), eager and
# graph-replayed, summarised per step by scripts/graph_trace.py (kernel busy time, gaps between
# kernels, overlap of the two streams).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05/graph; mkdir -p $O
LOSS=${LOSS:-l1}
for mode in eager graph; do
  extra=""; [ $mode = graph ] && extra="--inv-graph"
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/$mode -o run -- \
    python3 bench.py --no-cpu-baseline --no-configs --steps 2 --warmup 1 --inv-steps 10 --inv-loss $LOSS $extra \
    > $O/$mode.log 2>&1 || { echo "$mode trace failed"; tail -5 $O/$mode.log; exit 1; }
  echo "$mode traced"
done
python3 scripts/graph_trace.py $O/eager $O/graph | tee $O/summary.txt; rm -rf $O/eager_$LOSS $O/graph_$LOSS; mv $O/eager $O/eager_$LOSS; mv $O/graph $O/graph_$LOSS; mkdir -p $O/graph
find $O -name "*kernel_trace.csv" -size +20M -delete
