#!/bin/bash
# rocprofv3 kernel trace + HBM counters of the default bench (separate --pmc passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r01}
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-inversion ${BENCH_EXTRA:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 || exit $?
tail -1 $OUT/trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $BENCH > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $BENCH > $OUT/write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -20
# per-dispatch traces are large; the stats / counter summaries are what gets kept
find $OUT -name "*kernel_trace.csv" -delete
