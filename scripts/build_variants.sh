#!/bin/bash
# Build A/B variants of the HIP library next to the product build (CPU; hipcc cross-compiles):
#   scripts/build_variants.sh NAME "-DKNOB=V ..." [NAME "-D..."]...  -> nfi/libnfi_hip_NAME.so
# NAME "git:REV" builds the sources of git revision REV instead.
set -e
cd "$(dirname "$0")/.."
C=nerf-from-image_amd/csrc; O=nerf-from-image_amd/nfi
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -w"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  src=$C
  if [[ "$defs" == git:* ]]; then
    d=/tmp/nfi_variant_$name; rm -rf $d; mkdir -p $d
    git archive "${defs#git:}" $C include | tar -x -C $d
    src=$d/$C; defs=""
  fi
  /opt/rocm/bin/hipcc $FL $defs -o $O/libnfi_hip_$name.so $src/nfi_rays.hip $src/nfi_render.hip $src/nfi_producer.hip $src/nfi_conv.hip $(ls $src/nfi_gemm.hip 2>/dev/null) &
done
wait
