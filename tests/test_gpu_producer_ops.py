"""The producer's fused HIP operators (csrc/nfi_producer.hip via nfi/producer_ops.py) against
plain PyTorch fp32 formulations of the same ops — forward values and gradients (autograd of
the torch formulation) at the resolutions the synthesis network uses and odd channel counts."""

import math

import pytest
import torch
import torch.nn.functional as F

from oracle import producer_oracle as po
from nfi import producer, producer_ops

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')
GAIN = math.sqrt(2.0)


def _rand(*shape, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(shape, generator=g, device=DEV)


def _close(a, b, rel=2e-6):
    scale = float(b.abs().max()) + 1e-30
    err = float((a - b).abs().max())
    assert err <= rel * scale * 8, (err, scale)


def _act_ref(o, d, bias):
    x = o * d[:, :, None, None]
    x = (x + bias[None, :, None, None]) * GAIN
    return F.leaky_relu(x, 0.2)


@pytest.mark.parametrize('B,C,H', [(2, 3, 4), (2, 5, 8), (3, 7, 32), (2, 4, 128)])
def test_scale(B, C, H):
    x = _rand(B, C, H, H, seed=1).requires_grad_()
    s = _rand(B, C, seed=2).requires_grad_()
    g = _rand(B, C, H, H, seed=3)
    y = producer_ops.scale(x, s)
    y.backward(g)
    xr, sr = x.detach().clone().requires_grad_(), s.detach().clone().requires_grad_()
    (xr * sr[:, :, None, None]).backward(g)
    _close(y.detach(), (xr * sr[:, :, None, None]).detach())
    _close(x.grad, xr.grad)
    _close(s.grad, sr.grad, rel=1e-5)


@pytest.mark.parametrize('B,C,H', [(2, 3, 4), (2, 5, 8), (3, 7, 32), (2, 4, 128)])
def test_act(B, C, H):
    o = _rand(B, C, H, H, seed=4).requires_grad_()
    d = (_rand(B, C, seed=5).abs() + 0.1).requires_grad_()
    bias = 0.3 * _rand(C, seed=6)
    g = _rand(B, C, H, H, seed=7)
    y = producer_ops.act(o, d, bias, GAIN)
    y.backward(g)
    orf, drf = o.detach().clone().requires_grad_(), d.detach().clone().requires_grad_()
    yr = _act_ref(orf, drf, bias)
    yr.backward(g)
    _close(y.detach(), yr.detach())
    _close(o.grad, orf.grad)
    _close(d.grad, drf.grad, rel=1e-5)


@pytest.mark.parametrize('B,C,n', [(2, 3, 2), (2, 5, 4), (3, 6, 16), (2, 4, 64)])
def test_fir_up_act(B, C, n):
    t = _rand(B, C, 2 * n + 1, 2 * n + 1, seed=8).requires_grad_()
    d = (_rand(B, C, seed=9).abs() + 0.1).requires_grad_()
    bias = 0.3 * _rand(C, seed=10)
    g = _rand(B, C, 2 * n, 2 * n, seed=11)
    y = producer_ops.fir_up_act(t, d, bias, GAIN)
    y.backward(g)
    trf, drf = t.detach().clone().requires_grad_(), d.detach().clone().requires_grad_()
    o = po._depthwise(trf, producer.blur_kernel().to(DEV) * 4, stride=1, transpose=False)
    yr = _act_ref(o, drf, bias)
    yr.backward(g)
    _close(y.detach(), yr.detach())
    _close(t.grad, trf.grad)
    _close(d.grad, drf.grad, rel=1e-5)


@pytest.mark.parametrize('B,Ci,Co,n', [(1, 8, 4, 1), (2, 16, 8, 2), (3, 32, 24, 5), (2, 64, 32, 16),
                                        (1, 512, 256, 8)])
def test_up_conv(B, Ci, Co, n):
    """GEMM over the 9 taps + scatter == conv_transpose2d(x, w^T, stride=2) (fp64 reference:
    err <= 4x MIOpen's fp32 error, floor 1e-6 of the max), and its data gradient."""
    x = _rand(B, Ci, n, n, seed=16).requires_grad_()
    w = _rand(Co, Ci, 3, 3, seed=17) / (3 * Ci ** 0.5)
    g = _rand(B, Co, 2 * n + 1, 2 * n + 1, seed=18)
    t = producer_ops.up_conv(x, w)
    t.backward(g)
    x64 = x.detach().double().requires_grad_()
    r64 = F.conv_transpose2d(x64, w.double().transpose(0, 1), stride=2)
    r64.backward(g.double())
    r32 = F.conv_transpose2d(x.detach(), w.transpose(0, 1), stride=2)
    assert t.shape == r64.shape
    r64 = r64.detach()
    s = float(r64.abs().max())
    err, err32 = float((t.detach().double() - r64).abs().max()), float((r32.double() - r64).abs().max())
    assert err <= max(1e-6 * s, 4 * err32), (err, err32, s)
    gs = float(x64.grad.abs().max())
    assert float((x.grad.double() - x64.grad).abs().max()) <= 2e-6 * gs
    # a weight that takes gradients goes to MIOpen's transposed convolution (same values)
    wg = w.clone().requires_grad_()
    tg = producer_ops.up_conv(x.detach(), wg).detach()
    assert float((tg.double() - r64).abs().max()) <= max(1e-6 * s, 4 * err32)


@pytest.mark.parametrize('B,Ci,Co,n', [(2, 16, 8, 32), (1, 32, 16, 64), (2, 24, 8, 4), (2, 64, 32, 32)])
def test_up_conv_act_fused_matches_two_kernel_path(B, Ci, Co, n):
    """The fused scatter + FIR + epilogue kernel (2n % 64 == 0) matches up_conv then fir_up_act
    (the same operations; the compiler's FMA contraction may differ by an ulp), and so do the
    gradients (same backward kernels); n = 4 takes the unfused path.  Co = 32 at n = 32: the data
    gradient W9^T dP on the split GEMM, its scale from the maxima the fused backward pass leaves
    (nfi_syn_up_conv_act_backward_max) on one path and from a maximum pass over dP on the other."""
    x = _rand(B, Ci, n, n, seed=23).requires_grad_()
    w = _rand(Co, Ci, 3, 3, seed=24) / (3 * Ci ** 0.5)
    d = (_rand(B, Co, seed=25).abs() + 0.1).requires_grad_()
    bias = 0.3 * _rand(Co, seed=26)
    g = _rand(B, Co, 2 * n, 2 * n, seed=27)
    y = producer_ops.up_conv_act(x, w, d, bias, GAIN)
    y.backward(g)
    x2, d2 = x.detach().clone().requires_grad_(), d.detach().clone().requires_grad_()
    y2 = producer_ops.fir_up_act(producer_ops.up_conv(x2, w), d2, bias, GAIN)
    y2.backward(g)
    _close(y.detach(), y2.detach(), rel=1e-7)
    _close(x.grad, x2.grad, rel=1e-7)
    _close(d.grad, d2.grad, rel=1e-7)


@pytest.mark.parametrize('B,C,O,H', [(1, 8, 3, 2), (2, 32, 96, 4), (3, 512, 96, 16), (2, 128, 96, 128)])
def test_modulated_conv1x1(B, C, O, H):
    """bmm(W * s_b, x) == conv2d(x * s, W) for the 1x1 to-planes layers; d x and d s (fp64
    reference, 4x the fp32 torch formulation's error, floor 2e-6 of the max)."""
    x = _rand(B, C, H, H, seed=19).requires_grad_()
    s = _rand(B, C, seed=20).requires_grad_()
    w = _rand(O, C, 1, 1, seed=21) / C ** 0.5
    g = _rand(B, O, H, H, seed=22)
    y = producer_ops.modulated_conv1x1(x, s, w)
    y.backward(g)
    x64, s64 = x.detach().double().requires_grad_(), s.detach().double().requires_grad_()
    y64 = F.conv2d(x64 * s64[:, :, None, None], w.double())
    y64.backward(g.double())
    x32, s32 = x.detach().clone().requires_grad_(), s.detach().clone().requires_grad_()
    y32 = F.conv2d(x32 * s32[:, :, None, None], w)
    y32.backward(g)
    for got, ref, r32 in ((y.detach(), y64.detach(), y32.detach()), (x.grad, x64.grad, x32.grad),
                          (s.grad, s64.grad, s32.grad)):
        m = float(ref.abs().max())
        err, err32 = float((got.double() - ref).abs().max()), float((r32.double() - ref).abs().max())
        assert err <= max(2e-6 * m, 4 * err32), (err, err32, m)


@pytest.mark.parametrize('B,C,n', [(2, 3, 2), (2, 5, 4), (1, 96, 16), (2, 96, 128)])
@pytest.mark.parametrize('with_img', [True, False])
def test_up_add(B, C, n, with_img):
    img = _rand(B, C, n, n, seed=12).requires_grad_() if with_img else None
    c = _rand(B, C, 2 * n, 2 * n, seed=13).requires_grad_()
    bias = 0.3 * _rand(C, seed=14)
    g = _rand(B, C, 2 * n, 2 * n, seed=15)
    out = producer_ops.up_add(img, c, bias)
    out.backward(g)
    crf = c.detach().clone().requires_grad_()
    yr = crf + bias[None, :, None, None]
    if with_img:
        irf = img.detach().clone().requires_grad_()
        yr = po._depthwise(irf, producer.blur_kernel().to(DEV) * 4, stride=2, transpose=True) + yr
    yr.backward(g)
    _close(out.detach(), yr.detach())
    _close(c.grad, crf.grad)
    if with_img:
        _close(img.grad, irf.grad)


@pytest.mark.parametrize('B,C,n', [(2, 96, 2), (1, 96, 16), (2, 8, 64)])
@pytest.mark.parametrize('with_img', [True, False])
def test_up_add_channels_last(B, C, n, with_img):
    """The channels-last skip path (the producer's texel-major planes) == the NCHW one, values and
    gradients, and the 1x1 layer's channels-last output == its NCHW output."""
    img = _rand(B, C, n, n, seed=28).requires_grad_() if with_img else None
    c = _rand(B, C, 2 * n, 2 * n, seed=29).requires_grad_()
    bias = 0.3 * _rand(C, seed=30)
    g = _rand(B, C, 2 * n, 2 * n, seed=31)
    out = producer_ops.up_add(img, c, bias)
    out.backward(g)
    il = img.detach().to(memory_format=torch.channels_last).requires_grad_() if with_img else None
    cl = c.detach().to(memory_format=torch.channels_last).requires_grad_()
    out_l = producer_ops.up_add(il, cl, bias)
    assert out_l.is_contiguous(memory_format=torch.channels_last)
    out_l.backward(g.to(memory_format=torch.channels_last))
    _close(out_l.detach(), out.detach(), rel=1e-7)
    _close(cl.grad, c.grad, rel=1e-7)
    if with_img:
        _close(il.grad, img.grad, rel=1e-7)
    x = _rand(B, 16, 2 * n, 2 * n, seed=32)
    s = _rand(B, 16, seed=33)
    w = _rand(C, 16, 1, 1, seed=34)
    y0 = producer_ops.modulated_conv1x1(x, s, w)
    y1 = producer_ops.modulated_conv1x1(x, s, w, layout='nhwc')
    assert y1.is_contiguous(memory_format=torch.channels_last)
    _close(y1, y0, rel=1e-6)
    if C % 32 == 0:
        # the last layer: to-planes output as [B, C/32, 32, H, W] -> up_add writes texel-major
        # planes ([B, C/32, H, W, 32] storage); values and gradients as the NCHW chain
        xs = x.clone().requires_grad_()
        ss = s.clone().requires_grad_()
        y5 = producer_ops.modulated_conv1x1(xs, ss, w, layout='planes')
        p5 = producer_ops.up_add(il.detach().requires_grad_() if with_img else None, y5, bias)
        assert p5.dim() == 5 and p5.permute(0, 1, 3, 4, 2).is_contiguous()
        x0, s0 = x.clone().requires_grad_(), s.clone().requires_grad_()
        i0 = img.detach().clone().requires_grad_() if with_img else None
        p0 = producer_ops.up_add(i0, producer_ops.modulated_conv1x1(x0, s0, w), bias)
        _close(p5.reshape(p0.shape), p0.detach(), rel=1e-6)
        g5 = g.view(B, C // 32, 32, 2 * n, 2 * n).permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)
        p5.backward(g5)
        p0.backward(g)
        _close(xs.grad, x0.grad, rel=1e-6)
        _close(ss.grad, s0.grad, rel=1e-5)


def test_backends_agree_on_gpu():
    """Full producer: nfi's (Winograd F(4,3) 3x3 convolutions, fused epilogues) and the reference's
    op sequence (oracle/producer_oracle.py over the same modules, fp32) against that op sequence in
    float64 on the device.  d ws is ill-conditioned (sums over 2 x 96 x 256^2 plane gradients with
    cancellation): the reference's fp32 formulation itself is off by ~5e-4; nfi must stay within
    4x of that (the GPU parity convention of tests/test_gpu_parity.py)."""
    import copy
    from oracle.producer_oracle import ReferenceProducer
    torch.manual_seed(3)
    gen = producer.InversionGenerator(1.4).to(DEV).requires_grad_(False)
    ws = (0.6 * _rand(2, 15, 512, seed=16))
    g = _rand(2, 3, 32, 256, 256, seed=17)

    def ev(gn, dtype, be):
        gn = ReferenceProducer(gn) if be == 'torch' else gn
        w = ws.to(dtype).detach().clone().requires_grad_()
        planes, pal = gn.planes_and_palette(w)
        ((planes * g.to(dtype)).sum() + pal.sum()).backward()
        return planes.detach().double(), w.grad.double()

    ref = ev(copy.deepcopy(gen).double(), torch.float64, 'torch')
    err = {}
    for be in ('torch', 'hip'):
        p, d = ev(gen, torch.float32, be)
        err[be] = (float((p - ref[0]).abs().max() / ref[0].abs().max()), float((d - ref[1]).norm() / ref[1].norm()))
    print('vs fp64 (planes max/max, d ws rel L2):', err)
    assert err['hip'][0] < max(4 * err['torch'][0], 1e-5)
    assert err['hip'][1] < max(4 * err['torch'][1], 1e-4)
