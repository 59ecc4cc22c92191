#!/bin/bash
# Bench the product library and experiment builds (nfi/libnfi_hip_<variant>.so) back to back.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in nerf-from-image_amd/nfi/libnfi_hip*.so; do
  case "$lib" in *stamps*) continue;; esac
  NFI_LIBRARY=$PWD/$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inversion > gpurun_out/abl.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/abl.log; exit 1; }
  python -c "
import json,sys; d=json.loads(open('gpurun_out/abl.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['stages'].items()})" "$lib"
done
