set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -q --timeout 200 --timeout-method thread -rf -s > gpurun_out/gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; grep -E "passed|failed|FAILED|Error|split16 " gpurun_out/gemm_tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm_bench.log; exit 1; }
cat gpurun_out/gemm_bench.log | grep -v amdgpu.ids
