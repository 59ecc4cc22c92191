#!/bin/bash
# SQ counter passes (one rocprofv3 run per pass) on a short bench; kernels of nfi only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctr_${TAG:-r01}
mkdir -p $OUT
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-inversion ${BENCH_EXTRA:-}"
i=0
run() {
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $1 --kernel-include-regex 'nfi::' --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
}
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
run "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"
run "TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"

run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY"
ls $OUT
