export TMPDIR=/tmp
mkdir -p gpurun_out/lds
for p in 1 0; do
  POSE=$p timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex 'nfi::' --output-format csv -d gpurun_out/lds/p$p -o run -- python3 scripts/lds_probe.py 3 > gpurun_out/lds/p$p.log 2>&1 || { echo "pass $p failed"; tail -5 gpurun_out/lds/p$p.log; exit 1; }
done
echo done
