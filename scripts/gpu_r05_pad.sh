#!/bin/bash
# Round 5: (1) the round-4 padded-texel variant reconstructed (NFI_TEX_ROW_PAD=40, ATen-form grid
# gradients NFI_TILE_GG=0) under the -DNFI_TILE_CHECK build, ONCE; (2) padded layouts with the
# product's grid-gradient form, parity tests once each; (3) the RCCL test; (4) one LDS counter pass
# per layout (SQ_LDS_BANK_CONFLICT of tile_kernel); (5) an A/B bench of the layouts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
step() {   # step NAME SECONDS CMD...: continue after test failures (rc 1), stop on anything worse
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 $O/$name.log
  if grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault\|HSA_STATUS_ERROR" $O/$name.log; then
    echo "GPU fault in $name: stopping"; exit 3
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit 4; fi
}
PT="python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -rf -p no:cacheprovider"
step chkpadgg0 240 env NFI_LIBRARY=$L/libnfi_hip_chkpadgg0.so $PT tests/test_gpu_parity.py
for v in pad40 pad16 pad8; do
  step par_$v 240 env NFI_LIBRARY=$L/libnfi_hip_$v.so $PT tests/test_gpu_parity.py
done
step rccl 300 $PT tests/test_gpu_rccl.py
for v in default pad40 pad16 pad8; do
  if [ $v = default ]; then lib=$L/libnfi_hip.so; else lib=$L/libnfi_hip_$v.so; fi
  NFI_LIBRARY=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
    --kernel-include-regex 'tile_kernel' --output-format csv -d $O/lds_$v -o run -- python3 scripts/lds_probe.py 3 \
    > $O/lds_$v.log 2>&1 || { echo "lds pass $v failed"; tail -5 $O/lds_$v.log; exit 5; }
  echo "lds $v ok"
done
python3 - <<'EOF'
import csv, glob, collections
for v in ('default', 'pad40', 'pad16', 'pad8'):
    fs = glob.glob(f'gpurun_out/r05/lds_{v}/**/*counter_collection.csv', recursive=True)
    acc = collections.defaultdict(list)
    for f in fs:
        for r in csv.DictReader(open(f)):
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
    print(v, {k: f'{sum(x)/len(x):.3e}' for k, x in acc.items()})
EOF
for v in pad40 pad16 pad8; do
  step ab_$v 400 bash scripts/ab_bench.sh $L/libnfi_hip_$v.so 2 --steps 20 --warmup 5
done
echo done
