"""Per-layer times of the Winograd convolution paths on the LPIPS VGG16 shapes (64 images of 128^2):
fused kernel vs three-pass (transforms + hipBLASLt batched GEMM) vs MIOpen, forward with the VGG
epilogue.  Usage (GPU box): python scripts/wino_layers.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from nfi import conv  # noqa: E402

LAYERS = [(64, 64, 128), (64, 128, 64), (128, 128, 64), (128, 256, 32), (256, 256, 32),
          (256, 512, 16), (512, 512, 16), (512, 512, 8)]


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
    dev = torch.device('cuda:0')
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    tot = [0.0, 0.0, 0.0]
    for ci, co, hw in LAYERS:
        x = torch.randn(N, ci, hw, hw, device=dev)
        w = torch.randn(co, ci, 3, 3, device=dev) / (3 * ci ** .5)
        b = torch.randn(co, device=dev) * 0.1
        Uw, _ = conv.weights(w)
        res = []
        for fused in (True, False):
            conv.FUSED, conv.FUSED_MAX_CI, conv.FUSED_MAX_CO = fused, 1 << 20, 1 << 20
            res.append(timeit(lambda: conv._winograd(x, Uw, b, False)))
        conv.FUSED, conv.FUSED_MAX_CI, conv.FUSED_MAX_CO = True, 64, 64
        # the three-pass form with hipBLASLt's fp32 GEMM instead of the split-f16 product
        conv.FUSED, conv.SPLIT16 = False, False
        t_bmm = timeit(lambda: conv._winograd(x, Uw, b, False))
        conv.FUSED, conv.SPLIT16 = True, True
        print(f'    three-pass with hipBLASLt bmm {t_bmm:.3f} ms', flush=True)
        res.append(timeit(lambda: F.relu(F.conv2d(x, w, b, padding=1))))
        gf = 2 * 9 * ci * co * hw * hw * N / 4 / 1e9       # Winograd GEMM GFLOP (4x fewer products)
        print(f'{ci:4d}->{co:4d} @{hw:3d}: fused {res[0]:.3f} ms ({gf / res[0]:.0f} TF)  three-pass {res[1]:.3f} ms  '
              f'miopen+relu {res[2]:.3f} ms', flush=True)
        for i in range(3):
            tot[i] += res[i]
    print(f'total: fused {tot[0]:.3f}  three-pass {tot[1]:.3f}  miopen {tot[2]:.3f} ms')


if __name__ == '__main__':
    main()
