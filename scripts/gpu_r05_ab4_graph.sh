#!/bin/bash
# Round 5: the branch-free VOP2 entry form (NFI_TILE_AB=4) once through the parity file and, if
# green and fault-free, A/B against the product; then eager-vs-graph kernel traces of the inversion
# step (scripts/graph_trace.sh, l1 and vgg).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
PT="python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -rf -p no:cacheprovider"
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault\|HSA_STATUS_ERROR" "$@"; }
timeout -k 10 240 env NFI_LIBRARY=$L/libnfi_hip_ab4.so $PT tests/test_gpu_parity.py > $O/par_ab4.log 2>&1
rc=$?; echo "par_ab4 rc=$rc"; tail -3 $O/par_ab4.log
if fault $O/par_ab4.log; then echo "fault: stop"; exit 3; fi
if [ $rc -eq 0 ]; then
  timeout -k 10 500 bash scripts/ab_bench.sh $L/libnfi_hip_ab4.so 3 --steps 20 --warmup 5 > $O/ab_ab4.log 2>&1
  rc=$?; echo "ab_ab4 rc=$rc"; cat $O/ab_ab4.log
  if fault gpurun_out/ab_old.log gpurun_out/ab_new.log; then echo "fault: stop"; exit 3; fi
  [ $rc -eq 0 ] || exit $rc
fi
for loss in l1 vgg; do
  LOSS=$loss timeout -k 10 700 bash scripts/graph_trace.sh > $O/graph_$loss.log 2>&1
  rc=$?; echo "graph_$loss rc=$rc"; tail -4 $O/graph_$loss.log
  mv $O/graph/summary.txt $O/graph_summary_$loss.txt 2>/dev/null
  [ $rc -eq 0 ] || exit $rc
done
echo done
