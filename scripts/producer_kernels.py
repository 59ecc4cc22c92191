"""Roofline of the producer / loss HIP kernels (include/nfi_producer.h) at the largest shapes of
one inversion step (B images of the 256^2 synthesis block, LPIPS relu1_2 of 16·B copies at 128^2):
HIP-event time per launch on the launch stream, algorithmic HBM bytes per launch, GB/s and the
fraction of 8 TB/s.  Usage (GPU box): python scripts/producer_kernels.py [B] > profiles/...md"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
import torch  # noqa: E402

from nfi import producer_ops as po  # noqa: E402

PEAK = 8000.0


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape):
        return torch.randn(shape, device=dev, generator=g)

    C, n = 128, 128                       # b256.conv0: 256 -> 128 channels, 128^2 -> 256^2
    rows = []
    t = rnd(B, C, 2 * n + 1, 2 * n + 1)
    d, bias = rnd(B, C).abs() + 0.5, rnd(C)
    o = torch.empty(B, C, 2 * n, 2 * n, device=dev)
    y = torch.empty_like(o)
    P = B * C
    lib = po._lib.load()
    st = po._stream(dev)
    T2, O2 = (2 * n + 1) ** 2, (2 * n) ** 2
    rows.append(('fir_up_act (b256.conv0 tail)', timed(lambda: lib.nfi_syn_fir_up_act_forward(
        po._p(t), po._p(d), po._p(bias), po._p(o), po._p(y), P, C, n, po.ctypes.c_float(1.41), st)),
        4 * P * (T2 + 2 * O2)))
    gt = torch.empty_like(t)
    rows.append(('fir_up_bwd (adjoint FIR)', timed(lambda: lib.nfi_syn_fir_up_backward(
        po._p(o), po._p(gt), P, n, st)), 4 * P * (O2 + T2)))
    dd = torch.empty(B, C, device=dev)
    go = torch.empty_like(o)
    rows.append(('act_fwd (b256.conv1 epilogue)', timed(lambda: lib.nfi_syn_act_forward(
        po._p(o), po._p(d), po._p(bias), po._p(y), P, C, O2, po.ctypes.c_float(1.41), st)),
        4 * P * 2 * O2))
    rows.append(('act_bwd (+ d dcoefs)', timed(lambda: lib.nfi_syn_act_backward(
        po._p(y), po._p(o), po._p(d), po._p(bias), po._p(go), po._p(dd), P, C, O2,
        po.ctypes.c_float(1.41), st)), 4 * P * 3 * O2))
    rows.append(('scale_bwd (modulation backward)', timed(lambda: lib.nfi_syn_scale_backward(
        po._p(y), po._p(o), po._p(d), po._p(go), po._p(dd), P, O2, st)), 4 * P * 3 * O2))
    Pi = B * 96
    img = rnd(B, 96, n, n)
    c = rnd(B, 96, 2 * n, 2 * n)
    out = torch.empty_like(c)
    b96 = rnd(96)
    rows.append(('up_add (skip image, 96 ch)', timed(lambda: lib.nfi_syn_up_add_forward(
        po._p(img), po._p(c), po._p(b96), po._p(out), Pi, 96, n, st)), 4 * Pi * (n * n + 2 * O2)))
    gi = torch.empty_like(img)
    rows.append(('up_bwd', timed(lambda: lib.nfi_syn_up_backward(po._p(c), po._p(gi), Pi, n, st)),
                 4 * Pi * (O2 + n * n)))
    N, Cl, H = 16 * B, 64, 128            # LPIPS relu1_2 of the 16 copies
    f0, f1 = rnd(N, Cl, H, H).relu(), rnd(N, Cl, H, H).relu()
    w = rnd(Cl).abs()
    lo = torch.empty(N, device=dev)
    i0, i1 = torch.empty(N * H * H, device=dev), torch.empty(N * H * H, device=dev)
    rows.append(('lpips_fwd (relu1_2, 2 passes)', timed(lambda: lib.nfi_lpips_head_forward(
        po._p(f0), po._p(f1), po._p(w), po._p(lo), po._p(i0), po._p(i1), N, Cl, H * H, st)),
        4 * N * Cl * H * H * 2))
    gf = torch.empty_like(f0)
    gl = torch.ones(N, device=dev)
    rows.append(('lpips_bwd (relu1_2)', timed(lambda: lib.nfi_lpips_head_backward(
        po._p(gl), po._p(f0), po._p(f1), po._p(w), po._p(i0), po._p(i1), po._p(gf), N, Cl, H * H, st)),
        4 * N * Cl * H * H * 3))
    print(f'# producer / loss kernels, B={B} (largest shapes of one inversion step)\n')
    print('algorithmic bytes = compulsory reads + writes once each (re-reads of the 4x4 FIR halo, the')
    print('second pass of the LPIPS head and the stencil neighbours are cache traffic, not counted)\n')
    print('| kernel | µs/launch | MB/launch | GB/s | of 8 TB/s |')
    print('|---|---|---|---|---|')
    for name, sec, nbytes in rows:
        gbs = nbytes / sec / 1e9
        print(f'| {name} | {sec * 1e6:.1f} | {nbytes / 1e6:.1f} | {gbs:.0f} | {gbs / PEAK:.2f} |')


if __name__ == '__main__':
    main()
