"""The synthesis up-sampling convolutions (stride-2 3x3 transposed conv, stylegan.py:99-103) on
MIOpen vs one GEMM over all 9 taps (P = W9 [9*Co, Ci] @ x [Ci, n^2] per image) plus the tap
scatter into the (2n+1)^2 output.  Usage (GPU box): python scripts/upconv_probe.py [B]"""
import sys

import torch
import torch.nn.functional as F

LAYERS = [(512, 512, 4), (512, 512, 8), (512, 512, 16), (512, 512, 32), (512, 256, 64), (256, 128, 128)]


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


def scatter(P, n):
    B, _, Co = P.shape[:3]
    t = P.new_zeros(B, Co, 2 * n + 1, 2 * n + 1)
    for ky in range(3):
        for kx in range(3):
            t[:, :, ky:ky + 2 * n:2, kx:kx + 2 * n:2] += P[:, ky * 3 + kx]
    return t


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device('cuda:0')
    tot = [0.0, 0.0, 0.0, 0.0]
    for ci, co, n in LAYERS:
        x = torch.randn(B, ci, n, n, device=dev)
        w = torch.randn(co, ci, 3, 3, device=dev) / (3 * ci ** .5)
        wt = w.transpose(0, 1)
        W9 = w.permute(2, 3, 0, 1).reshape(9 * co, ci).contiguous()
        ref = F.conv_transpose2d(x.double(), wt.double(), stride=2)
        got = scatter(torch.matmul(W9, x.view(B, ci, n * n)).view(B, 9, co, n, n), n)
        mio = F.conv_transpose2d(x, wt, stride=2)
        s = float(ref.abs().max())
        e_g, e_m = float((got - ref).abs().max()) / s, float((mio - ref).abs().max()) / s
        t_m = timeit(lambda: F.conv_transpose2d(x, wt, stride=2))
        t_g = timeit(lambda: torch.matmul(W9, x.view(B, ci, n * n)))
        gf = 2 * 9 * ci * co * n * n * B / 1e9
        print(f'{ci:4d}->{co:4d} n={n:3d}: miopen {t_m:.3f} ms ({gf / t_m:.0f} TF)  gemm9 {t_g:.3f} ms '
              f'({gf / t_g:.0f} TF)  err miopen {e_m:.1e} gemm9 {e_g:.1e}', flush=True)
        tot[0] += t_m
        tot[1] += t_g
        # the data gradient: stride-2 convolution (MIOpen) vs im2col (F.unfold) + one GEMM
        gt = torch.randn(B, co, 2 * n + 1, 2 * n + 1, device=dev)
        wr = wt.reshape(ci, co * 9)
        ref_b = F.conv2d(gt.double(), wt.double(), stride=2)
        got_b = torch.matmul(wr, F.unfold(gt, 3, stride=2)).view(B, ci, n, n)
        e_b = float((got_b - ref_b).abs().max()) / float(ref_b.abs().max())
        tb_m = timeit(lambda: F.conv2d(gt, wt, stride=2))
        tb_u = timeit(lambda: F.unfold(gt, 3, stride=2))
        tb_g = timeit(lambda: torch.matmul(wr, F.unfold(gt, 3, stride=2)))
        print(f'   bwd: miopen {tb_m:.3f} ms ({gf / tb_m:.0f} TF)  unfold {tb_u:.3f} + gemm = {tb_g:.3f} ms  '
              f'err {e_b:.1e}', flush=True)
        tot[2] += tb_m
        tot[3] += tb_g
    print(f'total: miopen {tot[0]:.3f} ms  gemm9 (no scatter) {tot[1]:.3f} ms; bwd miopen {tot[2]:.3f} '
          f'unfold+gemm {tot[3]:.3f} ms')


if __name__ == '__main__':
    main()
