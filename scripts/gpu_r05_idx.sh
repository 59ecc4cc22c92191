#!/bin/bash
# Round 5: the VGPR-indexing probe (scripts/ubench/gpr_idx_probe.hip, built on the CPU), one run per
# pattern in its own process under a time limit, then (if nothing faulted) the eager-vs-graph traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault\|HSA_STATUS_ERROR\|HIP error" "$@"; }
for p in 0 5 1 4 6 2 3; do
  timeout -k 10 60 scripts/ubench/gpr_idx_probe 2048 $p > $O/idx_p$p.log 2>&1
  rc=$?; cat $O/idx_p$p.log
  if [ $rc -ne 0 ] || fault $O/idx_p$p.log; then echo "pattern $p rc=$rc: stopping"; exit 3; fi
done
if [ "${GRAPH:-1}" = 1 ]; then
  for loss in l1 vgg; do
    LOSS=$loss timeout -k 10 700 bash scripts/graph_trace.sh > $O/graph_$loss.log 2>&1
    rc=$?; echo "graph_$loss rc=$rc"; tail -4 $O/graph_$loss.log
    mv $O/graph/summary.txt $O/graph_summary_$loss.txt 2>/dev/null
    [ $rc -eq 0 ] || exit $rc
  done
fi
echo done
