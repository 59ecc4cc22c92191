"""The fused LPIPS distance head (HIP) against the torch formulation of the same op, and the
'vgg' inversion loss (LPIPS over 16 augmented copies, run.py:2211-2235) running through the HIP
path.  Parity against the reference is UNPINNED (no lpips package / weights offline; see
tests/test_lpips.py)."""

import pytest
import torch

from nfi import inversion, lpips, producer_ops

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


@pytest.mark.parametrize('N,C,H', [(3, 64, 32), (2, 512, 8), (5, 7, 3)])
def test_lpips_head_matches_torch(N, C, H):
    g = torch.Generator(device=DEV).manual_seed(C)
    f0 = torch.randn((N, C, H, H), device=DEV, generator=g).relu().requires_grad_()
    f1 = torch.randn((N, C, H, H), device=DEV, generator=g).relu()
    f0.data[0, :, 0, 0] = 0          # an all-zero feature vector (the a == 0 branch)
    w = torch.rand((C,), device=DEV, generator=g)
    gout = torch.randn((N,), device=DEV, generator=g)
    out = producer_ops.lpips_head(f0, f1, w)
    out.backward(gout)
    r0 = f0.detach().clone().requires_grad_()
    ref = (lpips.normalize(r0) - lpips.normalize(f1)).square().mul(w[None, :, None, None]).sum(1).mean((1, 2))
    ref.backward(gout)
    torch.testing.assert_close(out.detach(), ref.detach(), rtol=1e-5, atol=1e-7)
    gref = torch.nan_to_num(r0.grad, nan=0.0)     # torch: 0/0 at the all-zero vector
    torch.testing.assert_close(f0.grad, gref, rtol=1e-4, atol=1e-6 * float(gref.abs().max()))


@pytest.mark.parametrize('pool', [False, True])
@pytest.mark.parametrize('N,C,H,W', [(2, 64, 16, 16), (3, 5, 6, 12), (1, 512, 8, 8)])
def test_vgg_epilogue_matches_torch(N, C, H, W, pool):
    """bias + ReLU (+ MaxPool2d(2, 2)) of the VGG trunk: forward bit-exact against the torch ops,
    backward (tap gradient + pooled gradient) against autograd, including tied windows (all-zero
    after the ReLU, and equal positive values: the gradient goes to the first maximum)."""
    g = torch.Generator(device=DEV).manual_seed(N * C + H)
    x = torch.randn((N, C, H, W), device=DEV, generator=g)
    x[:, :, :2, :2] = 0.25                  # a window of equal positive values
    x[:, :, 2:4, :2] = -3.0                 # an all-zero window after the ReLU
    bias = torch.randn((C,), device=DEV, generator=g) * 0.1
    bias[0] = 0.0
    gy = torch.randn((N, C, H, W), device=DEV, generator=g)
    xa = x.clone().requires_grad_()
    out = producer_ops.vgg_epilogue(xa, bias, pool)
    xr = x.clone().requires_grad_()
    yr = torch.relu(xr + bias[None, :, None, None])
    if pool:
        gm = torch.randn((N, C, H // 2, W // 2), device=DEV, generator=g)
        mr = torch.nn.functional.max_pool2d(yr, 2, 2)
        y, m = out
        assert torch.equal(y, yr) and torch.equal(m, mr)
        torch.autograd.backward([y, m], [gy, gm])
        torch.autograd.backward([yr, mr], [gy, gm])
    else:
        assert torch.equal(out, yr)
        out.backward(gy)
        yr.backward(gy)
    assert torch.equal(xa.grad, xr.grad)


def test_lpips_backends_agree():
    torch.manual_seed(0)
    net = lpips.LPIPS(backend='torch').to(DEV)
    a = torch.tanh(torch.randn(4, 3, 128, 128, device=DEV)).requires_grad_()
    b = torch.tanh(torch.randn(4, 3, 128, 128, device=DEV))
    ref = net(a, b)
    ref.sum().backward()
    ga = a.grad.clone()
    a.grad = None
    net.backend = 'hip'
    out = net(a, b)
    out.sum().backward()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-6)
    assert float((a.grad - ga).norm() / ga.norm()) < 1e-4


def test_vgg_inversion_loss_runs():
    from test_producer import inversion_setup
    gen, d, meta, cfg = inversion_setup(DEV)
    cfg.steps, cfg.loss = 2, 'vgg'
    net = lpips.LPIPS().to(DEV)
    res = inversion.invert(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg, lpips_net=net)
    assert len(res.losses) == 2 and all(torch.isfinite(torch.tensor(res.losses)))
    assert torch.isfinite(res.ws).all()


def test_vgg_target_on_side_stream_matches_inline():
    """The target half of the 'vgg' loss (grid + target features) computed on a side stream gives
    the inline loss and gradient (same device draws, same kernels); the inversion
    trajectory with overlap_target on and off agrees in its losses (its latents differ only by
    the float-atomic order of d planes, amplified by Adam's normalised first steps)."""
    torch.manual_seed(0)
    net = lpips.LPIPS().to(DEV)
    rgb = torch.tanh(torch.randn(2, 64, 64, 3, device=DEV)).requires_grad_()
    target = torch.tanh(torch.randn(2, 64, 64, 3, device=DEV))
    torch.manual_seed(5)
    ref = inversion.image_loss('vgg', rgb, target, net)
    ref.backward()
    g_ref = rgb.grad.clone()
    rgb.grad = None
    torch.manual_seed(5)
    side = torch.cuda.Stream(device=DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        prepared = inversion.vgg_target('vgg', target, net)
    torch.cuda.current_stream(DEV).wait_stream(side)
    got = inversion.image_loss('vgg', rgb, target, net, prepared=prepared)
    got.backward()
    # (the distance head's spatial mean and grid_sample's backward accumulate with float atomics:
    #  reproducible to accumulation order, not bit for bit)
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=0.0)
    torch.testing.assert_close(rgb.grad, g_ref, rtol=1e-5, atol=1e-6 * float(g_ref.abs().max()))

    from test_producer import inversion_setup
    gen, d, meta, cfg = inversion_setup(DEV)
    cfg.steps, cfg.loss = 3, 'vgg'
    losses = []
    for overlap in (True, False):
        cfg.overlap_target = overlap
        torch.manual_seed(11)
        losses.append(inversion.invert(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg,
                                       lpips_net=net).losses)
    torch.testing.assert_close(torch.tensor(losses[0]), torch.tensor(losses[1]), rtol=1e-5, atol=1e-7)
