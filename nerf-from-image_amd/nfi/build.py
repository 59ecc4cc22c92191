"""Build the in-tree HIP library nfi/libnfi_hip.so for gfx950 (hipcc cross-compiles without a GPU)."""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), 'csrc')
OUT = os.path.join(HERE, 'libnfi_hip.so')
SOURCES = ['nfi_rays.hip', 'nfi_render.hip', 'nfi_producer.hip', 'nfi_conv.hip', 'nfi_gemm.hip', 'nfi_dconv.hip']
HEADERS = ['nfi_common.h', 'nfi_host.h']
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-shared', '-munsafe-fp-atomics',
         '-Wall', '-Wno-unused-result']


RENDER_SOURCES = ['nfi_rays.hip', 'nfi_render.hip', 'nfi_common.h', 'nfi_host.h']


def source_digest() -> str:
    """sha256 (16 hex) of the sources the renderer's kernels are built from (csrc/nfi_rays.hip,
    nfi_render.hip, their headers and include/nfi.h): stamps profiler counter files
    (profiles/latest_counters.json, renderer kernels) so bench.py can tell whether they describe
    the kernels it runs.  The caller-side operators (producer, Winograd) are not part of it."""
    import hashlib
    h = hashlib.sha256()
    inc = os.path.join(os.path.dirname(os.path.dirname(HERE)), 'include')
    for path in [os.path.join(CSRC, s) for s in RENDER_SOURCES] + [os.path.join(inc, 'nfi.h')]:
        with open(path, 'rb') as fh:
            h.update(os.path.basename(path).encode() + b'\0' + fh.read())
    return h.hexdigest()[:16]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    inc = os.path.join(os.path.dirname(os.path.dirname(HERE)), 'include')
    deps += [os.path.join(inc, h) for h in ('nfi.h', 'nfi_producer.h')]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


TORCH_OPS_SRC = os.path.join(CSRC, 'nfi_torch.cpp')
TORCH_OPS_OUT = os.path.join(HERE, 'libnfi_torch.so')


def build_torch_ops(force: bool = False, verbose: bool = True) -> str:
    """nfi/libnfi_torch.so: the TORCH_LIBRARY(nfi, ...) operators (csrc/nfi_torch.cpp) over the C-ABI,
    host C++ only (g++ against torch's headers and libraries), linked to nfi/libnfi_hip.so by rpath
    $ORIGIN; loaded with torch.ops.load_library (nfi.torch_ops)."""
    deps = [TORCH_OPS_SRC, OUT, os.path.join(os.path.dirname(os.path.dirname(HERE)), 'include', 'nfi.h')]
    if (not force and os.path.exists(TORCH_OPS_OUT)
            and all(os.path.getmtime(d) <= os.path.getmtime(TORCH_OPS_OUT) for d in deps if os.path.exists(d))):
        return TORCH_OPS_OUT
    import torch
    ti = os.path.dirname(torch.__file__)
    abi = int(torch.compiled_with_cxx11_abi())
    cmd = [os.environ.get('CXX', 'g++'), '-O2', '-std=c++17', '-fPIC', '-shared', TORCH_OPS_SRC, '-o',
           TORCH_OPS_OUT + '.tmp', f'-I{ti}/include', f'-I{ti}/include/torch/csrc/api/include', '-I/opt/rocm/include',
           '-D__HIP_PLATFORM_AMD__=1', '-DUSE_ROCM=1', f'-D_GLIBCXX_USE_CXX11_ABI={abi}', f'-L{ti}/lib', '-lc10',
           '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_hip', f'-L{HERE}', '-lnfi_hip', "-Wl,-rpath,$ORIGIN",
           f'-Wl,-rpath,{ti}/lib']
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(TORCH_OPS_OUT + '.tmp', TORCH_OPS_OUT)
    return TORCH_OPS_OUT


def build(force: bool = False, verbose: bool = True, variant: str = '') -> str:
    """variant 'stamps': profiling library libnfi_hip_stamps.so with per-phase cycle counters
    (-DNFI_STAMPS, loaded via NFI_LIBRARY by scripts/stamps.py); 'tilecheck': the tile pass's
    integrity-check build libnfi_hip_tilecheck.so (-DNFI_TILE_CHECK=1, tests/test_gpu_tile_check.py);
    never the product build."""
    out = OUT if not variant else OUT.replace('.so', f'_{variant}.so')
    if not force and not variant and not _stale():
        return out
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    extra = {'': [], 'stamps': ['-DNFI_STAMPS'], 'tilecheck': ['-DNFI_TILE_CHECK=1']}.get(variant)
    if extra is None:   # experiment builds: 'D<NAME>=<value>' -> -D<NAME>=<value>
        extra = ['-' + variant] if variant.startswith('D') else []
    cmd = [hipcc] + FLAGS + extra + ['-o', out + '.tmp'] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + '.tmp', out)
    return out


if __name__ == '__main__':
    var = ''
    if '--stamps' in sys.argv:
        var = 'stamps'
    for a in sys.argv:
        if a.startswith('--variant='):
            var = a.split('=', 1)[1]
    build(force='--force' in sys.argv, variant=var)
    if not var:
        build_torch_ops(force='--force' in sys.argv)
