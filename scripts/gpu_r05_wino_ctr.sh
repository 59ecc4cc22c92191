#!/bin/bash
# Round 5: SQ counters of the fused Winograd kernel (scripts/wino_layers.py's layers), two --pmc
# passes, each its own run: where the matrix cores' idle time goes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_wino; mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" --kernel-include-regex 'fused_kernel' --output-format csv \
      -d $OUT/$name -o run -- python3 scripts/wino_layers.py > $OUT/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$name.log; exit $rc; }
}
run sqa --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sqb --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
run sqc --pmc SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE
echo done
