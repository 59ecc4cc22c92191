"""Probe: MIOpen 3x3 convolution times of the LPIPS-VGG trunk (64 images of 128^2, the vgg loss's
16 x B=4 copies) vs the batched GEMMs a Winograd F(m,3) formulation would run on the matrix
cores (torch.bmm -> hipBLASLt, fp32): is a Winograd-on-MFMA convolution worth building?
Usage (GPU box): python scripts/wino_probe.py"""
import time

import torch
import torch.nn.functional as F

LAYERS = [(64, 64, 128), (64, 128, 64), (128, 128, 64), (128, 256, 32), (256, 256, 32),
          (256, 512, 16), (512, 512, 16), (512, 512, 8)]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    dev = torch.device('cuda:0')
    N = 64
    tot = {'conv': 0., 'dgrad': 0., 'w2': 0., 'w4': 0., 'w6': 0.}
    for cin, cout, hw in LAYERS:
        x = torch.randn(N, cin, hw, hw, device=dev)
        w = torch.randn(cout, cin, 3, 3, device=dev) / (3 * cin ** .5)
        gy = torch.randn(N, cout, hw, hw, device=dev)
        tc = timeit(lambda: F.conv2d(x, w, None, 1, 1))
        td = timeit(lambda: torch.nn.grad.conv2d_input(x.shape, w, gy, 1, 1))
        flops = 2 * 9 * cin * cout * hw * hw * N
        row = f'{cin:4d}->{cout:4d} @{hw:3d}: conv {tc:.3f} ms ({flops / tc / 1e9:.0f} TF-eq)  dgrad {td:.3f} ms'
        tot['conv'] += tc
        tot['dgrad'] += td
        for m in (2, 4, 6):
            a = m + 2
            P = N * ((hw + m - 1) // m) ** 2
            U = torch.randn(a * a, cout, cin, device=dev)
            V = torch.randn(a * a, cin, P, device=dev)
            tb = timeit(lambda: torch.bmm(U, V))
            gf = 2 * a * a * cout * cin * P
            row += f'  F({m},3) bmm {tb:.3f} ms ({gf / tb / 1e9:.0f} TF, {flops / tb / 1e9:.0f} TF-eq)'
            tot[f'w{m}'] += tb
        print(row, flush=True)
    print('totals ms:', {k: round(v, 3) for k, v in tot.items()})


if __name__ == '__main__':
    main()
