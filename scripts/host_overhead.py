"""Host cost of the pieces of one producer-op call (python + ctypes + torch allocator), to see
what an eager inversion step spends per custom launch.  Usage (GPU box): python scripts/host_overhead.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

from nfi import _lib, ops, producer_ops  # noqa: E402


def per_call(fn, n=20000):
    for _ in range(100):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    dev = torch.device('cuda:0')
    lib = _lib.load()
    o = torch.randn(4, 64, 16, 16, device=dev)
    d = torch.randn(4, 64, device=dev)
    b = torch.randn(64, device=dev)
    rows = [
        ('torch.cuda.current_stream(dev)', lambda: torch.cuda.current_stream(dev)),
        ('ops._stream(dev)', lambda: ops._stream(dev)),
        ('ctypes.c_void_p(ptr)', lambda: ctypes.c_void_p(12345)),
        ('t.data_ptr()', lambda: o.data_ptr()),
        ('_lib.load()', lambda: _lib.load()),
        ('getattr(lib, name)', lambda: getattr(lib, 'nfi_syn_act_forward')),
        ('t.contiguous()', lambda: o.contiguous()),
        ('torch.empty_like(t)', lambda: torch.empty_like(o)),
        ('ops._require_device(3)', lambda: ops._require_device(o, d, b)),
        ('lib.nfi_abi_version()', lambda: lib.nfi_abi_version()),
    ]
    y = torch.empty_like(o)
    s = ops._stream(dev)
    P, C, HW = 4 * 64, 64, 256
    fn = lib.nfi_syn_act_forward
    pp = [ctypes.c_void_p(t.data_ptr()) for t in (o, d, b, y)]
    rows.append(('raw ctypes launch (pre-built args)', lambda: fn(*pp, P, C, HW, ctypes.c_float(1.0), s)))
    rows.append(('act via _call', lambda: producer_ops._call(
        'nfi_syn_act_forward', producer_ops._p(o), producer_ops._p(d), producer_ops._p(b), producer_ops._p(y),
        P, C, HW, ctypes.c_float(1.0), ops._stream(dev))))
    with torch.no_grad():
        rows.append(('producer_ops.act (no grad)', lambda: producer_ops.act(o, d, b, 1.0)))
    og = o.clone().requires_grad_()
    rows.append(('producer_ops.act (grad graph)', lambda: producer_ops.act(og, d, b, 1.0)))
    rows.append(('torch mul (grad graph)', lambda: og * 2.0))
    rows.append(('torch mul (no grad)', lambda: o * 2.0))
    for name, f in rows:
        us = per_call(f)
        torch.cuda.synchronize()
        print(f'{name:40s} {us:7.2f} us', flush=True)


if __name__ == '__main__':
    main()
