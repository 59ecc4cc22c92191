"""The fused LPIPS distance head (HIP) against the torch formulation of the same op, and the
'vgg' inversion loss (LPIPS over 16 augmented copies, run.py:2211-2235) running through the HIP
path.  Parity against the reference is UNPINNED (no lpips package / weights offline; see
tests/test_lpips.py)."""

import pytest
import torch

from oracle import producer_oracle as po
from nfi import inversion, lpips, producer_ops

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


@pytest.mark.parametrize('N,C,H', [(3, 64, 32), (2, 512, 8), (5, 7, 3), (2, 128, 5), (4, 256, 16), (64, 64, 128)])
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
    ref = (po.lpips_normalize(r0) - po.lpips_normalize(f1)).square().mul(w[None, :, None, None]).sum(1).mean((1, 2))
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


def _lpips_eval(net, a, b):
    a = a.detach().clone().requires_grad_()
    out = net(a, b)
    out.sum().backward()
    return out.detach().double().cpu(), a.grad.double().cpu()


def test_lpips_backends_agree():
    """nfi.lpips (Winograd F(4,3) trunk, fused epilogues and distance head) and the same with the
    MIOpen trunk against an fp64 evaluation of the reference formulation (oracle/producer_oracle.py
    over the same parameters); that formulation in fp32 (MIOpen) is measured beside them.  The Winograd trunk's fp32 transform rounding (a few 1e-6
    per layer, tests/test_gpu_conv.py) compounds over 13 layers and the ReLU masks to ~2e-4 in
    the image gradient: about 10x the MIOpen path's, still fp32-grade."""
    import copy
    torch.manual_seed(0)
    from oracle import producer_oracle as po
    net = lpips.LPIPS().to(DEV)
    a = torch.tanh(torch.randn(4, 3, 128, 128, device=DEV))
    b = torch.tanh(torch.randn(4, 3, 128, 128, device=DEV))
    net64 = copy.deepcopy(net).double().cpu()
    ref, gref = _lpips_eval(po.ReferenceLPIPS(net64), a.double().cpu(), b.double().cpu())

    def errs(r):
        return float((r[0] - ref).abs().max() / ref.abs().max()), float((r[1] - gref).norm() / gref.norm())

    e_torch = errs(_lpips_eval(po.ReferenceLPIPS(net), a, b))
    e_wino = errs(_lpips_eval(net, a, b))
    try:
        lpips.VGG16Features.winograd = False
        e_miopen = errs(_lpips_eval(net, a, b))
    finally:
        lpips.VGG16Features.winograd = True
    print(f'vs fp64 (loss, image gradient): torch fp32 {e_torch}, hip+miopen {e_miopen}, hip+winograd {e_wino}')
    assert e_miopen[0] < 1e-5 and e_miopen[1] < max(4 * e_torch[1], 1e-5)
    assert e_wino[0] < 1e-5 and e_wino[1] < 1e-3
    # where the Winograd gradient error sits: a forward near-tie (a 2x2 max-pool window or a ReLU
    # input within rounding of 0) decided the other way reroutes one feature gradient, a local
    # jump; elsewhere the gradient is as accurate as the forward
    g = _lpips_eval(net, a, b)[1]
    rel = ((g - gref).abs() / gref.abs().max()).flatten()
    q = torch.quantile(rel[torch.randperm(rel.numel())[:100000]], torch.tensor([0.5, 0.99, 0.999], dtype=rel.dtype))
    print('winograd |d image| error / max, quantiles 50/99/99.9 %:', q.tolist(),
          'share > 1e-4:', float((rel > 1e-4).double().mean()))
    assert float(q[1]) < 1e-5


def test_vgg_inversion_loss_runs():
    from test_producer import inversion_setup
    gen, d, meta, cfg = inversion_setup(DEV)
    cfg.steps, cfg.loss = 2, 'vgg'
    net = lpips.LPIPS().to(DEV)
    res = inversion.invert(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg, lpips_net=net)
    assert len(res.losses) == 2 and all(torch.isfinite(torch.tensor(res.losses)))
    assert torch.isfinite(res.ws).all()


@pytest.mark.parametrize('B,H,W,white,scale', [(2, 64, 64, False, None), (1, 32, 48, True, None),
                                                (4, 128, 128, False, None), (2, 40, 40, False, 0.3),
                                                (2, 40, 40, True, 3.0)])
def test_aug_sample_matches_grid_sample(B, H, W, white, scale):
    """The augmented copies (nfi_aug_sample_forward / _backward) against the reference's
    expand-to-15-copies + grid_sample(bilinear, zeros, align_corners=False) in fp64: values and
    the gradient summed over the copies (gathered, no atomics).  `scale` forces every copy's zoom
    (0.3: each output pixel's corners spread over ~3 input pixels; 3.0: many samples per pixel)."""
    g = torch.Generator(device=DEV).manual_seed(H + B)
    img = torch.tanh(torch.randn((B, H, W, 3), device=DEV, generator=g)).requires_grad_()
    grid = inversion.augment_grid((15 * B, 6, H, W), 1.0, DEV, generator=g)
    if scale is not None:       # rescale the affine maps about the centre
        grid = grid / scale
    gout = torch.randn((15 * B, 3, H, W), device=DEV, generator=g)
    out = producer_ops.aug_sample(img, grid, 15, white)
    out.backward(gout)
    i64 = img.detach().double().requires_grad_()
    ref = inversion.apply_grid(inversion._copies(i64.permute(0, 3, 1, 2)), grid.double(), white)
    ref.backward(gout.double())
    i32 = img.detach().clone().requires_grad_()
    r32 = inversion.apply_grid(inversion._copies(i32.permute(0, 3, 1, 2)), grid, white)
    r32.backward(gout)
    assert out.shape == ref.shape
    ref = ref.detach()
    # the fp32 source coordinates ((g + 1) W - 1) / 2 carry ~ulp(W) error: 4x torch fp32's own
    # error against fp64 (the GPU parity convention), floor 1e-6
    err, err32 = float((out.detach().double() - ref).abs().max()), float((r32.detach().double() - ref).abs().max())
    assert err <= max(1e-6, 4 * err32), (err, err32)
    gr = i64.grad
    gerr, gerr32 = float((img.grad.double() - gr).abs().max()), float((i32.grad.double() - gr).abs().max())
    assert gerr <= max(1e-6 * float(gr.abs().max()), 4 * gerr32), (gerr, gerr32)


@pytest.mark.parametrize('N,H,W', [(60, 128, 128), (3, 7, 5), (2, 1, 4), (1, 6, 1)])
def test_affine_grid_matches_aten(N, H, W):
    """nfi_aug_affine_grid (the augmentation's grid, run.py:749) against F.affine_grid(align_corners=
    False) on the same device: ATen's base grid and product order, so equal to an ulp of the grid's
    magnitude (the batched product's accumulation order is hipBLASLt's); sizes 1 included."""
    g = torch.Generator(device=DEV).manual_seed(N * 100 + H)
    theta = torch.randn((N, 2, 3), device=DEV, generator=g)
    ours = producer_ops.affine_grid(theta, [N, 6, H, W])
    ref = torch.nn.functional.affine_grid(theta, [N, 6, H, W], align_corners=False)
    assert ours.shape == ref.shape
    tol = 2.5e-7 * (1.0 + float(theta.abs().amax()) * 3)
    assert float((ours - ref).abs().max()) <= tol
    grid = inversion.augment_grid((4, 6, 16, 16), 1.0, DEV, generator=g)   # the inversion's call
    assert grid.shape == (4, 16, 16, 2) and torch.isfinite(grid).all()


@pytest.mark.parametrize('N,Co,H,W', [(2, 64, 16, 64), (3, 64, 32, 128), (1, 8, 48, 64)])
def test_vgg_first_layer(N, Co, H, W):
    """The fused first VGG layer (direct 3x3 conv + bias + ReLU; backward threshold + data gradient)
    against fp64 torch: within 4x the fp32 torch formulation's own error (floor 1e-6 of the max)."""
    g = torch.Generator(device=DEV).manual_seed(N * H + Co)
    x = torch.randn((N, 3, H, W), device=DEV, generator=g).requires_grad_()
    w = torch.randn((Co, 3, 3, 3), device=DEV, generator=g) * 0.3
    b = torch.randn((Co,), device=DEV, generator=g) * 0.1
    gy = torch.randn((N, Co, H, W), device=DEV, generator=g)
    y = producer_ops.vgg_first(x, w, b)
    y.backward(gy)
    x64 = x.detach().double().requires_grad_()
    y64 = torch.relu(torch.nn.functional.conv2d(x64, w.double(), b.double(), padding=1))
    y64.backward(gy.double())
    x32 = x.detach().clone().requires_grad_()
    y32 = torch.relu(torch.nn.functional.conv2d(x32, w, b, padding=1))
    y32.backward(gy)
    for got, ref, r32 in ((y.detach(), y64.detach(), y32.detach()), (x.grad, x64.grad, x32.grad)):
        m = float(ref.abs().max())
        err, err32 = float((got.double() - ref).abs().max()), float((r32.double() - ref).abs().max())
        assert err <= max(1e-6 * m, 4 * err32), (err, err32, m)


def test_vgg_first_layer_with_scaling_layer():
    """The LPIPS ScalingLayer folded into the first layer (lpips 0.1: (x - shift) / scale, then conv1_1 +
    ReLU): forward equal to the unfolded ops up to one rounding of the normalised input, and the image
    gradient through the division against fp64 torch."""
    g = torch.Generator(device=DEV).manual_seed(21)
    N, Co, H, W = 2, 64, 32, 64
    net = lpips.LPIPS().to(DEV)
    x = torch.rand((N, 3, H, W), device=DEV, generator=g) * 2 - 1
    w = torch.randn((Co, 3, 3, 3), device=DEV, generator=g) * 0.3
    b = torch.randn((Co,), device=DEV, generator=g) * 0.1
    gy = torch.randn((N, Co, H, W), device=DEV, generator=g)
    xa = x.clone().requires_grad_()
    y = producer_ops.vgg_first(xa, w, b, net.shift, net.scale)
    y.backward(gy)
    xb = x.clone().requires_grad_()
    yb = producer_ops.vgg_first((xb - net.shift) / net.scale, w, b)
    yb.backward(gy)
    assert float((y - yb).abs().max()) <= 1e-6 * float(yb.abs().max())
    x64 = x.double().requires_grad_()
    y64 = torch.relu(torch.nn.functional.conv2d((x64 - net.shift.double()) / net.scale.double(), w.double(),
                                                b.double(), padding=1))
    y64.backward(gy.double())
    m = float(x64.grad.abs().max())
    assert float((xa.grad.double() - x64.grad).abs().max()) <= 4 * max(
        float((xb.grad.double() - x64.grad).abs().max()), 1e-7 * m)


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
