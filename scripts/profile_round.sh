#!/bin/bash
# rocprofv3 evidence for one round: kernel trace + stats, HBM counters (FETCH_SIZE and WRITE_SIZE
# in separate passes, MI355X_MICROARCH.md §HBM) and SQ / TCC passes (issue, MFMA, LDS, waits, L2)
# of the headline bench config.  Each pass its own run, none combined with a trace domain.
# Summarise with: python scripts/summarize_round.py gpurun_out/prof_$TAG $TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-inversion --no-configs ${BENCH_EXTRA:-}"
run() {   # name, rocprofv3 args...
  local name=$1; shift
  echo "[profile] pass $name"
  timeout -s KILL ${PASS_TIMEOUT:-150} rocprofv3 "$@" --kernel-include-regex 'nfi::' --output-format csv \
      -d $OUT/$name -o run -- python3 $BENCH > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name failed rc=$rc"; tail -5 $OUT/$name.log; exit $rc; fi
}
echo "[profile] pass trace"
timeout -s KILL ${PASS_TIMEOUT:-150} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
    -- python3 $BENCH > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
tail -c 600 $OUT/trace.log
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sqa --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sqb --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_F16 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
run tcc --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
# per-dispatch traces are large; the stats / counter summaries are what gets kept
find $OUT -name "*kernel_trace.csv" -delete
echo "[profile] done"
