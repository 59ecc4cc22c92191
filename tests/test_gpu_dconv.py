"""The direct 3x3 convolution on the f16 matrix cores (nfi_dconv3x3, csrc/nfi_dconv.hip; nfi.conv's
form for the LPIPS 128^2 / 64^2 layers) against fp64 convolutions: forward, the VGG block epilogue
(bias, ReLU, 2x2 max pool), the data gradient with the ReLU mask in the staging, per-image operand
scales, and the dispatch through conv3x3 / vgg_block.  Bar: the largest error relative to the largest
output <= max(4 x MIOpen fp32's own, 2e-6) (split-f16 products: 3 2^-22 |a||b| each at worst)."""

import pytest
import torch
import torch.nn.functional as F

from nfi import conv

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')

SHAPES = [(2, 16, 64, 8, 64), (3, 64, 64, 16, 64), (2, 64, 128, 16, 128), (1, 128, 64, 8, 128),
          (2, 32, 192, 24, 64), (9, 48, 64, 8, 64)]


def _err(a, ref):
    ref = ref.detach()
    return float((a.detach().double().cpu() - ref).abs().max() / ref.abs().max())


def _wset(w):
    U, Ut = conv.weights(w)
    for ws in (U, Ut):    # (packed on first use)
        if ws.direct is None:
            w_, co, ci, flip = ws.direct_src
            ws.direct = conv._direct_pack(w_, co, ci, flip, conv._stream(w.device))
    assert U.direct is not None and Ut.direct is not None
    return U, Ut


@pytest.mark.parametrize('N,Ci,Co,H,W', SHAPES)
def test_dconv_forward(N, Ci, Co, H, W):
    g = torch.Generator(device=DEV).manual_seed(Ci * Co + H + N)
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    U, _ = _wset(w)
    y = conv._direct(x, U)
    yd = F.conv2d(x.double().cpu(), w.double().cpu(), padding=1)
    ym = F.conv2d(x, w, padding=1)
    e, em = _err(y, yd), _err(ym, yd)
    print(f'direct {e:.2e}, miopen {em:.2e}')
    assert e <= max(4 * em, 2e-6), (e, em)


@pytest.mark.parametrize('pool', [False, True])
@pytest.mark.parametrize('N,Ci,Co,H,W', [(2, 64, 64, 16, 64), (3, 32, 128, 8, 128)])
def test_dconv_vgg_epilogue(N, Ci, Co, H, W, pool):
    g = torch.Generator(device=DEV).manual_seed(N + Ci + Co + H + pool)
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    b = torch.randn((Co,), device=DEV, generator=g) * 0.1
    U, _ = _wset(w)
    out = conv._direct(x, U, b, pool)
    yd = torch.relu(F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), padding=1))
    y = out[0] if pool else out
    assert _err(y, yd) <= 2e-6
    if pool:
        assert out[1].shape == (N, Co, H // 2, W // 2)
        assert _err(out[1], F.max_pool2d(yd, 2, 2)) <= 2e-6


@pytest.mark.parametrize('masked', [False, True])
@pytest.mark.parametrize('N,C,Co,H,W', [(2, 64, 64, 16, 64), (2, 128, 64, 8, 128), (1, 64, 128, 8, 64)])
def test_dconv_data_gradient(N, C, Co, H, W, masked):
    """The flipped / transposed pack: conv3x3(g', w') = conv_transpose2d(g', w, padding=1), g' = g or,
    with relu_y, g where relu_y > 0 (threshold_backward in the staging)."""
    gen = torch.Generator(device=DEV).manual_seed(N * C + Co + H + masked)
    w = torch.randn((Co, C, 3, 3), device=DEV, generator=gen) / (3 * C ** 0.5)
    gy = torch.randn((N, Co, H, W), device=DEV, generator=gen)
    yv = torch.randn((N, Co, H, W), device=DEV, generator=gen) if masked else None
    _, Ut = _wset(w)
    gx = conv._direct(gy, Ut, relu_y=yv)
    gm = gy * (yv > 0) if masked else gy
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.double().cpu(), gm.double().cpu(), 1, 1)
    refm = torch.nn.grad.conv2d_input((N, C, H, W), w, gm, 1, 1)
    e, em = _err(gx, ref), _err(refm, ref)
    print(f'direct dgrad {e:.2e}, miopen {em:.2e}')
    assert e <= max(4 * em, 2e-6), (e, em)


@pytest.mark.parametrize('small', [1e-6, 1e-9])
def test_dconv_per_image_scale(small):
    """One image far below the others keeps its own precision, and its result equals the same image
    run alone bit for bit (its scale is its own: sharded = unsharded)."""
    N, Ci, Co, H, W = 4, 64, 64, 16, 64
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    x[2] *= small
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / (3 * Ci ** 0.5)
    U, _ = _wset(w)
    y = conv._direct(x, U)
    yd = F.conv2d(x[2:3].double().cpu(), w.double().cpu(), padding=1)
    assert _err(y[2:3], yd) <= 2e-6
    alone = conv._direct(x[2:3].contiguous(), U)
    assert torch.equal(alone, y[2:3])


def test_dconv_lpips_shape_against_miopen():
    """The LPIPS conv1_2 layer at full size (64 images of 128^2, 64 -> 64, bias, ReLU, pool) against
    MIOpen fp32 (both near fp32 rounding; relative to the largest output)."""
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.relu(torch.randn((64, 64, 128, 128), device=DEV, generator=g))
    w = torch.randn((64, 64, 3, 3), device=DEV, generator=g) / 24.0
    b = torch.randn((64,), device=DEV, generator=g) * 0.1
    U, _ = _wset(w)
    y, m = conv._direct(x, U, b, True)
    ym = torch.relu(F.conv2d(x, w, b, padding=1))
    scale = float(ym.abs().max())
    assert float((y - ym).abs().max()) <= 4e-6 * scale
    assert torch.equal(m, F.max_pool2d(y, 2, 2))


def test_dconv_dispatch_and_autograd(monkeypatch):
    """vgg_block / conv3x3 take the direct kernel on eligible shapes, forward and backward (the ReLU
    mask in the staging when there is no pool gradient), and match fp64 autograd."""
    calls = []
    real = conv._direct

    def spy(*a, **k):
        calls.append(a[0].shape)
        return real(*a, **k)

    monkeypatch.setattr(conv, '_direct', spy)
    g = torch.Generator(device=DEV).manual_seed(11)
    N, Ci, Co, H, W = 2, 64, 64, 64, 64
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / 24.0
    b = torch.randn((Co,), device=DEV, generator=g) * 0.1
    gy = torch.randn((N, Co, H, W), device=DEV, generator=g)
    xa = x.clone().requires_grad_()
    y = conv.vgg_block(xa, w, b, False)
    y.backward(gy)
    assert len(calls) == 2, calls    # forward + data gradient
    xd = x.double().cpu().requires_grad_()
    yd = torch.relu(F.conv2d(xd, w.double().cpu(), b.double().cpu(), padding=1))
    yd.backward(gy.double().cpu())
    assert _err(y, yd) <= 2e-6
    rel = float((xa.grad.double().cpu() - xd.grad).norm() / xd.grad.norm())
    assert rel < 1e-5, rel
    calls.clear()
    xb = x.clone().requires_grad_()
    conv.conv3x3(xb, w).backward(gy)
    assert len(calls) == 2, calls


def test_dconv_chained_maxima_equal_maxima_pass():
    """The per-image maxima a producer leaves on its output (the LPIPS first layer, a dconv VGG
    epilogue) give the next dconv the same scale as a maxima pass over that output: equal results, bit
    for bit; a modified tensor drops them."""
    from nfi import producer_ops
    g = torch.Generator(device=DEV).manual_seed(5)
    img = torch.randn((3, 3, 64, 64), device=DEV, generator=g)
    w1 = torch.randn((64, 3, 3, 3), device=DEV, generator=g) / 5.0
    b1 = torch.randn((64,), device=DEV, generator=g) * 0.1
    w2 = torch.randn((64, 64, 3, 3), device=DEV, generator=g) / 24.0
    b2 = torch.randn((64,), device=DEV, generator=g) * 0.1
    w3 = torch.randn((128, 64, 3, 3), device=DEV, generator=g) / 24.0
    U2, _ = _wset(w2)
    U3, _ = _wset(w3)
    with torch.no_grad():
        y1 = producer_ops.vgg_first(img, w1, b1)
        assert conv._maxima_of(y1) is not None
        y2, m2 = conv._direct(y1, U2, b2, True)
        y2r, m2r = conv._direct(y1.clone(), U2, b2, True)
        assert torch.equal(y2, y2r) and torch.equal(m2, m2r)
        assert conv._maxima_of(y2) is not None and conv._maxima_of(m2) is not None
        y3 = conv._direct(y2, U3, b2.repeat(2))
        assert torch.equal(y3, conv._direct(y2.clone(), U3, b2.repeat(2)))
        y2.mul_(2.0)
        assert conv._maxima_of(y2) is None


def test_dconv_modulated_forward_backward(monkeypatch):
    """modulated_conv3x3 (conv2d(x * s[:, :, None, None], w), stylegan.py:130) on the direct kernel: the
    scale folded into the staging (per-image maxima of |x s|), the backward as the direct data
    gradient + nfi_syn_scale_backward; against fp64 autograd."""
    calls = []
    real = conv._direct

    def spy(*a, **k):
        calls.append(k.get('scale') is not None)
        return real(*a, **k)

    monkeypatch.setattr(conv, '_direct', spy)
    monkeypatch.setattr(conv, 'DIRECT_MOD', True)
    g = torch.Generator(device=DEV).manual_seed(13)
    N, Ci, Co, H, W = 2, 64, 128, 64, 64
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    s = torch.rand((N, Ci), device=DEV, generator=g) * 1.5 + 0.25
    s[1] *= 1e-3
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / 24.0
    gy = torch.randn((N, Co, H, W), device=DEV, generator=g)
    xa, sa = x.clone().requires_grad_(), s.clone().requires_grad_()
    y = conv.modulated_conv3x3(xa, sa, w)
    y.backward(gy)
    assert calls == [True, False], calls
    xd, sd = x.double().cpu().requires_grad_(), s.double().cpu().requires_grad_()
    yd = F.conv2d(xd * sd[:, :, None, None], w.double().cpu(), padding=1)
    yd.backward(gy.double().cpu())
    for n in range(N):   # each image on its own scale
        assert _err(y[n], yd[n]) <= 2e-6, n
    assert float((xa.grad.double().cpu() - xd.grad).norm() / xd.grad.norm()) < 1e-5
    assert float((sa.grad.double().cpu() - sd.grad).norm() / sd.grad.norm()) < 1e-5


def test_dconv_vgg_block_pool_backward():
    """vgg_block with the pool on the direct path: the pool routing + ReLU backward leaves gz's per-image
    maxima for the direct data gradient (no maxima pass), against fp64 autograd."""
    g = torch.Generator(device=DEV).manual_seed(17)
    N, Ci, Co, H, W = 2, 64, 64, 64, 64
    x = torch.randn((N, Ci, H, W), device=DEV, generator=g)
    w = torch.randn((Co, Ci, 3, 3), device=DEV, generator=g) / 24.0
    b = torch.randn((Co,), device=DEV, generator=g) * 0.1
    gy = torch.randn((N, Co, H, W), device=DEV, generator=g)
    gm = torch.randn((N, Co, H // 2, W // 2), device=DEV, generator=g)
    xa = x.clone().requires_grad_()
    y, m = conv.vgg_block(xa, w, b, True)
    torch.autograd.backward([y, m], [gy, gm])
    xd = x.double().cpu().requires_grad_()
    yd = torch.relu(F.conv2d(xd, w.double().cpu(), b.double().cpu(), padding=1))
    md = F.max_pool2d(yd, 2, 2)
    torch.autograd.backward([yd, md], [gy.double().cpu(), gm.double().cpu()])
    assert _err(y, yd) <= 2e-6 and _err(m, md) <= 2e-6
    rel = float((xa.grad.double().cpu() - xd.grad).norm() / xd.grad.norm())
    assert rel < 1e-4, rel    # (a pool argmax can flip on a near-tie)
