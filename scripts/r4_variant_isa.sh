#!/bin/bash
# Rebuild round 4's padded tile-texel variant on the CPU from round 4's final
# sources (git d44ebd7) with its one change — tile rows of 8 texels padded by 40 floats (LDS 38,820 B) —
# next to that commit's product build, and report the tile kernel's DS address rewrites (isa_lint rule 3).
# Output: /tmp/r4var/{nfi_render,nfi_render_pad}.s
set -e
cd "$(dirname "$0")/.."
R=$PWD; D=/tmp/r4var; rm -rf $D; mkdir -p $D
git archive d44ebd7 nerf-from-image_amd/csrc include | tar -x -C $D
cd $D/nerf-from-image_amd/csrc
python3 - <<'PY'
s = open('nfi_render.hip').read()
s = s.replace('constexpr int TEXF = TTX * TTY * XS;            // 1,440 floats',
              'constexpr int TEXR = TTX * XS + 40;\nconstexpr int TEXF = TTY * TEXR;\n'
              '__device__ __forceinline__ int tex_at(int texel) { return (texel / TTX) * TEXR + (texel % TTX) * XS; }')
s = s.replace('''    const float* t = Tex + slot * XS + 4 * k;
    const float4 t00 = *reinterpret_cast<const float4*>(t);
    const float4 t01 = *reinterpret_cast<const float4*>(t + XS);
    const float4 t10 = *reinterpret_cast<const float4*>(t + TTX * XS);
    const float4 t11 = *reinterpret_cast<const float4*>(t + (TTX + 1) * XS);''', '''    const float* t = Tex + tex_at(slot) + 4 * k;
    const float4 t00 = *reinterpret_cast<const float4*>(t);
    const float4 t01 = *reinterpret_cast<const float4*>(t + XS);
    const float4 t10 = *reinterpret_cast<const float4*>(t + TEXR);
    const float4 t11 = *reinterpret_cast<const float4*>(t + TEXR + XS);''')
s = s.replace('*reinterpret_cast<float4*>(Tex + texel * XS + 4 * c4) = v;',
              '*reinterpret_cast<float4*>(Tex + tex_at(texel) + 4 * c4) = v;')
assert s.count('tex_at(') == 3
open('nfi_render_pad.hip', 'w').write(s)
PY
for f in nfi_render nfi_render_pad; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -w --cuda-device-only -S $f.hip -o $D/$f.s &
done
wait
cd $R
python3 - <<'PY'
import sys
sys.path[:0] = ['scripts', 'nerf-from-image_amd']
import isa_lint as L
for name in ('nfi_render', 'nfi_render_pad'):
    f = L.ds_addr_rewrites(f'/tmp/r4var/{name}.s', 2, 'tile_kernel')
    print(name, 'tile_kernel DS address rewrites within 2 wait states:', len(f))
    for x in f:
        print('   ', x[2], '->', x[3])
PY
