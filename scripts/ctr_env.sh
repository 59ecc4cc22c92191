#!/bin/bash
# HBM counters (FETCH_SIZE, WRITE_SIZE: separate passes) of the renderer bench under environment
# settings (ENVS as in ab_env.sh), summed per kernel by scripts/ctr_kernels.py.  GPU box.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in ${ENVS:--}; do
  name=$(echo "$e" | tr ',=' '__')
  out=gpurun_out/ctre_$name
  envs=(); [ "$e" != "-" ] && IFS=',' read -ra envs <<< "$e"
  for pass in FETCH_SIZE WRITE_SIZE; do
    env "${envs[@]}" timeout -s KILL 150 rocprofv3 --pmc $pass --kernel-include-regex 'nfi::' --output-format csv \
        -d $out/$pass -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-inversion \
        --no-configs > $out.$pass.log 2>&1 || { echo "ctr $name $pass failed"; tail -5 $out.$pass.log; exit 1; }
  done
  python scripts/ctr_kernels.py $out $name
done
