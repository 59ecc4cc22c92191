#!/bin/bash
# Round 6: the split GEMM with buffer-load staging (in-tree build) against the previous kernel
# (libnfi_hip_g0.so): GEMM / conv / producer / LPIPS tests, the per-shape bench of both, then the
# inversion legs of both (bench.py, renderer stages skipped from the comparison).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
L=$PWD/nerf-from-image_amd/nfi
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -x -rf -p no:cacheprovider \
  tests/test_gpu_gemm.py tests/test_gpu_conv.py tests/test_gpu_producer_ops.py tests/test_gpu_lpips.py > $O/gemmab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gemmab_tests.log; [ $rc -eq 0 ] || exit 3
GEMM_VARIANTS="22:0:1" timeout -k 10 300 python3 scripts/gemm_bench.py > $O/gemm_bench_new.log 2>&1 || exit 4
NFI_AB_OLDER=1 NFI_LIBRARY=$L/libnfi_hip_g0.so GEMM_VARIANTS="22:0:1" timeout -k 10 300 python3 scripts/gemm_bench.py > $O/gemm_bench_old.log 2>&1 || exit 5
paste -d'\n' $O/gemm_bench_new.log $O/gemm_bench_old.log | cut -c1-150
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 > $O/gemmab_inv_new.log 2>&1 || exit 6
  NFI_LIBRARY=$L/libnfi_hip_g0.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 5 --warmup 2 > $O/gemmab_inv_old.log 2>&1 || exit 7
  for f in new old; do python - $O/gemmab_inv_$f.log $f <<'PYEOF'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(sys.argv[2], {k: (d[k]['ms_per_step'], d[k]['rest_ms_per_step']) for k in ('inversion', 'inversion_l1')})
PYEOF
  done
done
