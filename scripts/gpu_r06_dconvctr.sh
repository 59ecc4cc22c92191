#!/bin/bash
# Round 6: counters of the direct convolution on one layer shape (one --pmc pass per run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_dconv${TAG:-}; mkdir -p $OUT
SHAPE=${SHAPE:-64 64 64 128}
timeout -k 10 120 python3 scripts/dconv_one.py $SHAPE 20 || exit 1
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" --kernel-include-regex 'dconv_kernel' --output-format csv \
      -d $OUT/$name -o run -- python3 scripts/dconv_one.py $SHAPE 10 > $OUT/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$name.log; exit $rc; }
}
run trace --kernel-trace --stats
run sqa --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sqb --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
run sqc --pmc SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
echo done
