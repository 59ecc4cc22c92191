"""HBM rate of the Winograd input / output transform kernels alone on the LPIPS-VGG16 layer
shapes (64 images of 128^2): bytes = x read + V written (input), M read + y written (output).
Usage (GPU box): python scripts/wino_transforms_bw.py [N]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

from nfi import _lib, ops  # noqa: E402

LAYERS = [(64, 128), (128, 64), (256, 32), (512, 16), (512, 8)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device('cuda:0')
    lib = _lib.load()
    st = ops._stream(dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for C, H in LAYERS:
        x = torch.randn(N, C, H, H, device=dev)
        P = N * (H // 4) ** 2
        V = torch.empty(36, C, P, device=dev)
        y = torch.empty_like(x)
        t_in = timeit(lambda: lib.nfi_wino_input_transform(p(x), p(V), N, C, H, H, st))
        t_out = timeit(lambda: lib.nfi_wino_output_transform(p(V), None, p(y), None, N, C, H, H, st))
        xb, vb = x.numel() * 4, V.numel() * 4
        print(f'C={C:3d} H={H:3d}: input {t_in * 1e3:7.1f} us {(xb + vb) / t_in / 1e6:6.0f} GB/s   '
              f'output {t_out * 1e3:7.1f} us {(xb + vb) / t_out / 1e6:6.0f} GB/s', flush=True)


if __name__ == '__main__':
    main()
