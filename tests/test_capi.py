"""CPU-side checks of the C-ABI boundary: the in-tree HIP library loads, exports every entry
point declared in include/*.h (nfi.h, nfi_producer.h), and the ctypes structs match the C layout (gcc-compiled
probe).  No compute calls (no GPU here)."""

import os
import re
import subprocess
import ctypes

import pytest

from nfi import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'nfi.h')
HEADERS = [os.path.join(ROOT, 'include', h) for h in sorted(os.listdir(os.path.join(ROOT, 'include')))
           if h.endswith('.h')]


def declared_functions():
    src = '\n'.join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r'^\s*(?:int32_t|int64_t|const char\*)\s+(nfi_\w+)\s*\(', src, re.M)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SIGNATURES), 'ctypes binding and header disagree'
    assert lib.nfi_abi_version() == _lib.ABI_VERSION


def test_decoder_size_constant_matches_header():
    src = open(HEADER).read()
    assert int(re.search(r'#define NFI_DEC_SIZE (\d+)', src).group(1)) == _lib.DEC_SIZE


@pytest.mark.parametrize('struct', ['nfi_camera', 'nfi_field', 'nfi_render_args', 'nfi_render_grad_args'])
def test_struct_layout_matches_c(tmp_path, struct):
    py = {'nfi_camera': _lib.NfiCamera, 'nfi_field': _lib.NfiField,
          'nfi_render_args': _lib.NfiRenderArgs, 'nfi_render_grad_args': _lib.NfiRenderGradArgs}[struct]
    fields = [f[0] for f in py._fields_]
    probe = tmp_path / 'probe.c'
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', 'int main(void){',
             f'printf("%zu\\n", sizeof({struct}));']
    lines += [f'printf("%zu\\n", offsetof({struct}, {f}));' for f in fields]
    lines += ['return 0;}']
    probe.write_text('\n'.join(lines))
    exe = tmp_path / 'probe'
    subprocess.run(['gcc', '-o', str(exe), str(probe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(py)
    for f, off in zip(fields, vals[1:]):
        assert getattr(py, f).offset == off, f


def test_bad_arguments_are_rejected_without_launch():
    lib = _lib.load()
    args = _lib.NfiRenderArgs()
    code = lib.nfi_render_forward(ctypes.byref(args), None)
    assert code == -1
    assert b'null' in lib.nfi_last_error()


def test_torch_ops_library_registers():
    """nfi/libnfi_torch.so (TORCH_LIBRARY(nfi, ...), csrc/nfi_torch.cpp) loads here without a GPU and
    registers every operator with its schema; a CPU tensor raises instead of computing."""
    import torch
    from nfi import torch_ops
    torch_ops.load()
    for name in torch_ops.OPS:
        assert hasattr(torch.ops.nfi, name), name
    schema = str(torch.ops.nfi.volume_render.default._schema)
    assert schema.startswith('nfi::volume_render(Tensor planes_tm, Tensor? palette, Tensor ro, Tensor rd')
    cu = torch.jit.CompilationUnit(torch_ops.render_script_source())
    assert 'nfi::volume_render' in str(cu.render_rays.graph)
    with pytest.raises(RuntimeError, match='HIP devices only'):
        torch.ops.nfi.cumprod_exclusive(torch.ones(2, 3))
