"""One split-f16 Winograd-product shape launched REPS times (for rocprofv3 counter passes on the GEMM
alone).  Usage: python scripts/gemm_one.py [Co Ci P [reps]]  (default: 128 128 16384, the LPIPS
conv2 products over 64 images)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd')]
import torch  # noqa: E402

from nfi import _lib, conv  # noqa: E402

DEV = torch.device('cuda:0')


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def main():
    Co, Ci, P = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (128, 128, 16384)))
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    lib = _lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    A = torch.randn((36, Co, Ci), device=DEV)
    B = torch.randn((36, Ci, P), device=DEV)
    hi = torch.empty(A.shape, device=DEV, dtype=torch.int16)
    lo = torch.empty(A.shape, device=DEV, dtype=torch.int16)
    inv = torch.empty((36,), device=DEV)
    slots = torch.zeros((conv.slot_words(),), device=DEV, dtype=torch.int32)
    _lib.check(lib.nfi_split16_pack(_p(A), 36, Co * Ci, _p(hi), _p(lo), _p(inv), st), 'pack')
    C = torch.empty((36, Co, P), device=DEV)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(reps + 2):
        if i == 2:
            e0.record()
        _lib.check(lib.nfi_absmax_slots(_p(B), 1, B.numel(), _p(slots), st), 'absmax')
        _lib.check(lib.nfi_gemm_split16(_p(hi), _p(lo), _p(inv), _p(B), _p(slots), _p(C), 36, Co, P, Ci, P, st),
                   'gemm')
    e1.record()
    torch.cuda.synchronize()
    fl = 2 * 36 * Co * Ci * P
    ms = e0.elapsed_time(e1) / reps
    print(f'Co {Co} Ci {Ci} P {P}: {ms:.3f} ms per (absmax + gemm), {fl / ms / 1e9:.1f} TF fp32-equivalent')


if __name__ == '__main__':
    main()
