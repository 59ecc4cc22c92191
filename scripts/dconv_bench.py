"""Per-layer timing of the LPIPS-shaped 3x3 convolutions: the direct split-f16 kernel (nfi_dconv3x3,
with its per-image maxima pass) against the Winograd forms (fused kernel / three-pass split GEMM)
and MIOpen fp32.  Forward with the VGG epilogue and the data gradient (ReLU-masked where the block
would mask it).  Usage: python scripts/dconv_bench.py  (one GPU)."""

import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'nerf-from-image_amd'))
from nfi import conv  # noqa: E402

DEV = torch.device('cuda:0')
LAYERS = [(64, 64, 64, 128), (64, 64, 128, 64), (64, 128, 128, 64), (64, 128, 256, 32)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    torch.backends.cudnn.allow_tf32 = False
    g = torch.Generator(device=DEV).manual_seed(0)
    for N, Ci, Co, H in LAYERS:
        x = torch.relu(torch.randn((N, Ci, H, H), device=DEV, generator=g))
        w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
        b = torch.randn((Co,), device=DEV, generator=g) * 0.1
        gy = torch.randn((N, Co, H, H), device=DEV, generator=g)
        yv = torch.randn((N, Co, H, H), device=DEV, generator=g)
        U, Ut = conv.weights(w)
        flops = 2.0 * N * Co * Ci * 9 * H * H
        row = [f'{N:3d}x{Ci:3d}->{Co:3d} @{H:3d}^2']
        if conv._direct_ok(U, x):
            t = timeit(lambda: conv._direct(x, U, b, True))
            row.append(f'direct fwd {t:.3f} ms ({flops / t / 1e9:.0f} TF)')
        if conv._direct_ok(Ut, gy):
            t = timeit(lambda: conv._direct(gy, Ut, relu_y=yv))
            row.append(f'direct dgrad {t:.3f} ms')
        t = timeit(lambda: conv._winograd(x, U, b, True))
        row.append(f'winograd fwd {t:.3f} ms')
        t = timeit(lambda: conv._winograd(gy * (yv > 0), Ut))
        row.append(f'winograd dgrad(+mask) {t:.3f} ms')
        t = timeit(lambda: torch.relu(F.conv2d(x, w, b, padding=1)))
        row.append(f'miopen fwd {t:.3f} ms')
        slots = torch.empty((conv.slot_words(),), device=DEV, dtype=torch.int32)
        t = timeit(lambda: conv._call('nfi_absmax_slots', x.data_ptr(), N, Ci * H * H, slots.data_ptr(),
                                      conv._stream(DEV)))
        row.append(f'(absmax {t:.3f} ms)')
        print('  '.join(row), flush=True)


if __name__ == '__main__':
    main()
