"""Winograd F(4x4, 3x3) convolutions (nfi.conv, csrc/nfi_conv.hip) against an fp64 convolution:
forward, the data gradient, and the fused VGG16 block epilogue.  Bar: the largest error relative
to the largest output is <= 2e-5 (F(4,3)'s fp32 transform rounding is a few 1e-6; MIOpen's error
on the same case is computed beside it for the record; TF32 is off in both, run.py:59-60)."""

import pytest
import torch
import torch.nn.functional as F

from nfi import conv

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')

SHAPES = [(2, 16, 24, 8, 8), (3, 64, 64, 16, 12), (2, 128, 96, 32, 32), (1, 512, 512, 8, 8),
          (2, 64, 64, 128, 128), (1, 32, 3, 4, 4)]


def _err(a, ref):
    ref = ref.detach()
    return float((a.detach().double().cpu() - ref).abs().max() / ref.abs().max())


@pytest.mark.parametrize('N,Ci,Co,H,W', SHAPES)
def test_winograd_conv_forward_and_data_gradient(N, Ci, Co, H, W):
    g = torch.Generator(device=DEV).manual_seed(Ci * Co + H)
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    gy = torch.randn((N, Co, H, W), device=DEV, generator=g)
    xa = x.clone().requires_grad_()
    y = conv.conv3x3(xa, w)
    y.backward(gy)
    xd = x.double().cpu().requires_grad_()
    yd = F.conv2d(xd, w.double().cpu(), padding=1)
    yd.backward(gy.double().cpu())
    xm = x.clone().requires_grad_()
    ym = F.conv2d(xm, w, padding=1)
    ym.backward(gy)
    e_w, e_m = _err(y, yd), _err(ym, yd)
    ge_w, ge_m = _err(xa.grad, xd.grad), _err(xm.grad, xd.grad)
    print(f'winograd {e_w:.2e} / {ge_w:.2e}, miopen {e_m:.2e} / {ge_m:.2e} (forward / data gradient)')
    assert e_w <= max(8 * e_m, 2e-5), (e_w, e_m)
    assert ge_w <= max(8 * ge_m, 2e-5), (ge_w, ge_m)


@pytest.mark.parametrize('pool', [False, True])
@pytest.mark.parametrize('N,Ci,Co,H', [(2, 64, 64, 16), (3, 128, 256, 8), (1, 16, 32, 4)])
def test_winograd_vgg_block(N, Ci, Co, H, pool):
    """relu(conv + b) (+ MaxPool2d(2, 2)) from the output transform; backward through the ReLU /
    pool routing and the data-gradient Winograd."""
    g = torch.Generator(device=DEV).manual_seed(N + Ci + H)
    x = torch.randn((N, Ci, H, H), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    b = torch.randn((Co,), device=DEV, generator=g) * 0.1
    xa = x.clone().requires_grad_()
    out = conv.vgg_block(xa, w, b, pool)
    xd = x.double().cpu().requires_grad_()
    yd = torch.relu(F.conv2d(xd, w.double().cpu(), b.double().cpu(), padding=1))
    gy = torch.randn((N, Co, H, H), device=DEV, generator=g)
    if pool:
        y, m = out
        md = F.max_pool2d(yd, 2, 2)
        gm = torch.randn(m.shape, device=DEV, generator=g)
        torch.autograd.backward([y, m], [gy, gm])
        torch.autograd.backward([yd, md], [gy.double().cpu(), gm.double().cpu()])
        assert _err(m, md) < 2e-5
    else:
        y = out
        y.backward(gy)
        yd.backward(gy.double().cpu())
    assert _err(y, yd) < 2e-5
    # the ReLU mask / pool argmax can flip on values within rounding of 0 / of a tie
    rel = float((xa.grad.double().cpu() - xd.grad).norm() / xd.grad.norm())
    assert rel < 1e-4, rel


@pytest.mark.parametrize('pool', [False, True])
@pytest.mark.parametrize('N,Ci,Co,H,W', [(3, 64, 64, 16, 12), (2, 8, 40, 8, 20), (1, 256, 96, 4, 4),
                                         (5, 128, 128, 32, 32)])
def test_fused_kernel_matches_three_pass(N, Ci, Co, H, W, pool):
    """The fused Winograd kernel (transforms + MFMA products in one pass) against the three-pass
    form (HIP transforms around hipBLASLt's batched GEMM): same transforms, different summation
    order of the products only.  Partial tile blocks (P % 32 != 0), Co not a multiple of 32."""
    g = torch.Generator(device=DEV).manual_seed(N * Ci + Co)
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    b = torch.randn((Co,), device=DEV, generator=g) * 0.1
    Uw, _ = conv.weights(w)
    assert Uw.packed is not None
    outs = []
    for fused in (True, False):
        conv.FUSED, conv.FUSED_MAX_CI, conv.FUSED_MAX_CO = fused, 1 << 20, 1 << 20
        try:
            r = conv._winograd(x, Uw, b if pool else None, pool)
        finally:
            conv.FUSED, conv.FUSED_MAX_CI, conv.FUSED_MAX_CO = True, 64, 64
        outs.append(r if pool else (r,))
    for a, ref in zip(*outs):
        scale = float(ref.abs().max())
        assert float((a - ref).abs().max()) <= 1e-5 * scale, float((a - ref).abs().max()) / scale


def test_weight_cache_follows_in_place_updates():
    w = torch.randn((32, 32, 3, 3), device=DEV)   # channel counts the split GEMM takes (multiples of 32)
    ws1, _ = conv.weights(w)
    U1, A1 = ws1.U, ws1.packed
    U1c, A1c = U1.clone(), A1.clone()
    assert conv.weights(w)[0].U is U1
    with torch.no_grad():
        w.mul_(2)
    ws2, _ = conv.weights(w)
    torch.testing.assert_close(ws2.U, 2 * U1c)
    torch.testing.assert_close(ws2.packed, 2 * A1c)
    # the split halves follow too: x2 is a power of two, so hi / lo are equal and the scale halves
    assert torch.equal(ws2.split[0], ws1.split[0]) and torch.equal(ws2.split[1], ws1.split[1])
    torch.testing.assert_close(ws2.split[2], ws1.split[2] * 2)


def test_trainable_weight_takes_the_library_path():
    """A weight that requires grad (training, not the inversion) gets its gradient from MIOpen;
    the fused VGG block refuses it."""
    x = torch.randn((1, 16, 8, 8), device=DEV)
    w = torch.randn((16, 16, 3, 3), device=DEV, requires_grad=True)
    conv.conv3x3(x, w).sum().backward()
    assert w.grad is not None
    with pytest.raises(NotImplementedError):
        conv.vgg_block(x, w, torch.zeros(16, device=DEV), False)


@pytest.mark.parametrize('N,C,Co,H', [(2, 128, 96, 16), (4, 512, 512, 4), (3, 16, 32, 8), (2, 64, 128, 32), (1, 128, 128, 64)])
def test_modulated_conv(N, C, Co, H):
    """conv2d(x * s, w) with the modulation folded into the input transform, against the fp64
    formulation: output, d x and d s (the synthesis layers' style gradient)."""
    g = torch.Generator(device=DEV).manual_seed(N + C + H)
    x = torch.randn((N, C, H, H), device=DEV, generator=g)
    s = torch.rand((N, C), device=DEV, generator=g) + 0.5
    w = torch.randn((Co, C, 3, 3), device=DEV, generator=g) / (3 * C ** 0.5)
    gy = torch.randn((N, Co, H, H), device=DEV, generator=g)
    xa, sa = x.clone().requires_grad_(), s.clone().requires_grad_()
    y = conv.modulated_conv3x3(xa, sa, w)
    y.backward(gy)
    xd, sd = x.double().cpu().requires_grad_(), s.double().cpu().requires_grad_()
    yd = F.conv2d(xd * sd[:, :, None, None], w.double().cpu(), padding=1)
    yd.backward(gy.double().cpu())
    assert _err(y, yd) < 2e-5
    assert _err(xa.grad, xd.grad) < 2e-5
    assert float((sa.grad.double().cpu() - sd.grad).norm() / sd.grad.norm()) < 1e-4


@pytest.mark.parametrize('epilogue', ['none', 'relu', 'pool'])
@pytest.mark.parametrize('N,Ci,Co,H,W', [(2, 64, 64, 32, 32), (1, 64, 128, 16, 48), (2, 32, 64, 16, 16),
                                         (1, 64, 64, 128, 128)])
def test_fused_split_kernel(N, Ci, Co, H, W, epilogue):
    """nfi_wino_conv_fused_split (the fused layers' products on the f16 matrix cores, the 36 products
    consumed row by row by the output transform) against an fp64 convolution + epilogue (the 2e-5
    bar) and against fused_kernel (fp32 MFMAs) on the same inputs."""
    g = torch.Generator(device=DEV).manual_seed(N + Ci + Co + H + W)
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    x[:, :, : H // 4] *= 1e-3                         # magnitudes spread inside a workgroup's region
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    b = 0.1 * torch.randn((Co,), device=DEV, generator=g)
    Uw, _ = conv.weights(w)
    assert Uw.split is not None
    bias = None if epilogue == 'none' else b
    pool = epilogue == 'pool'
    old = conv.FUSED_SPLIT, conv.FUSED_MAX_CO
    outs = {}
    try:
        conv.FUSED_MAX_CO = 1 << 20                      # (the fused path for every shape here)
        for mode in (True, False):
            conv.FUSED_SPLIT = mode
            outs[mode] = conv._winograd(x, Uw, bias, pool)
    finally:
        conv.FUSED_SPLIT, conv.FUSED_MAX_CO = old
    ref = F.conv2d(x.double(), w.double(), padding=1)
    if bias is not None:
        ref = torch.relu(ref + b.double()[None, :, None, None])
    refs = (ref, F.max_pool2d(ref, 2)) if pool else (ref,)
    for got_s, got_f, r in zip(outs[True] if pool else (outs[True],), outs[False] if pool else (outs[False],), refs):
        scale = float(r.abs().max())
        e_s = float((got_s.double() - r).abs().max()) / scale
        e_f = float((got_f.double() - r).abs().max()) / scale
        print(f'  split {e_s:.3g}  fused fp32 {e_f:.3g}')
        assert e_s <= 2e-5, (e_s, e_f)
