"""Size-independent properties at BASELINE's full p3d size (128², 64+64 samples, R=256 planes),
where the fp64 oracle is too slow to run: determinism, output bounds, linearity of the backward
in the upstream gradient, and exact linearity of the loss in the palette (rgb = sum_i w_i p_i·palette
is linear in it, so a directional difference equals <dL/dpalette, delta> up to fp32 rounding)."""

import pytest
import torch

import nfi
from gpu_helpers import rel_l2, synthetic_inputs

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def _render(inp, meta, seed, palette=None, g_scale=1.0, grads=True):
    nfi.configure(scene_range=float(meta['scene_range']), white_background=False, fine_sampling=True)
    planes = inp['planes'].to(DEV).requires_grad_(grads)
    pal = (inp['palette'] if palette is None else palette).to(DEV).requires_grad_(grads)
    cam = inp['cam'].to(DEV).requires_grad_(grads)
    focal = inp['focal'].to(DEV).requires_grad_(grads)
    f = nfi.TriplaneField(planes=planes, palette=pal, w1=inp['w1'].to(DEV), b1=inp['b1'].to(DEV),
                          w2=inp['w2'].to(DEV), b2=inp['b2'].to(DEV), alpha=1.0, beta=0.1)
    rgb, depth, mask, _, _, _ = nfi.render(f, int(meta['H']), int(meta['W']), cam, focal, None, None, None,
                                           int(meta['S']), randomize=True, seed=seed)
    out = {'rgb': rgb.detach(), 'depth': depth.detach(), 'mask': mask.detach()}
    if grads:
        g = torch.Generator(device='cpu').manual_seed(3)
        g_rgb = torch.randn(rgb.shape, generator=g).to(DEV) * g_scale
        g_mask = torch.randn(mask.shape, generator=g).to(DEV) * g_scale
        loss = (rgb * g_rgb).sum() + (mask * g_mask).sum()
        loss.backward()
        out.update(loss=loss.detach(), d_planes=planes.grad, d_palette=pal.grad, d_cam=cam.grad,
                   d_focal=focal.grad)
    return out


@pytest.fixture(scope='module')
def full():
    inp, meta = synthetic_inputs(B=2, H=128, W=128, S=64, R=256, scene_range=1.4, seed=77)
    return inp, meta


def test_forward_deterministic_and_bounded(full):
    inp, meta = full
    a = _render(inp, meta, seed=11, grads=False)
    b = _render(inp, meta, seed=11, grads=False)
    for k in ('rgb', 'depth', 'mask'):
        assert torch.equal(a[k], b[k]), k
    assert float(a['mask'].min()) >= 0.0 and float(a['mask'].max()) <= 1.0 + 1e-6
    assert float(a['depth'].min()) >= 0.0
    pal_max = float(inp['palette'].abs().max())
    assert float(a['rgb'].abs().max()) <= pal_max * (1 + 1e-6)
    assert float(a['mask'].mean()) > 0.05        # the field is not empty
    c = _render(inp, meta, seed=12, grads=False)
    assert not torch.equal(a['rgb'], c['rgb'])   # another Philox stream moves the samples


def test_backward_linear_in_upstream_gradient(full):
    inp, meta = full
    a = _render(inp, meta, seed=5)
    b = _render(inp, meta, seed=5, g_scale=2.0)
    # fixed-order reductions, exact in fp32 (x2 is exact through every product and sum): d palette,
    # and the pose gradients (per-entry grid gradients, per-ray sums, per-image segment sums)
    for k in ('d_palette', 'd_cam', 'd_focal'):
        assert torch.equal(b[k], 2 * a[k]), k
    # d planes: the tile bins are filled by cursor atomics, so the order of a tile's entries (and the
    # fp32 rounding of its register sums) varies run to run (determinism)
    assert rel_l2(b['d_planes'], 2 * a['d_planes']) < 1e-5


def test_loss_linear_in_palette(full):
    inp, meta = full
    base = _render(inp, meta, seed=9)
    delta = torch.randn(inp['palette'].shape, generator=torch.Generator().manual_seed(4))
    eps = 1e-2
    moved = _render(inp, meta, seed=9, palette=inp['palette'] + eps * delta, grads=True)
    lhs = float(moved['loss'] - base['loss'])
    rhs = eps * float((base['d_palette'].cpu() * delta).sum())
    assert abs(lhs - rhs) <= 1e-3 * abs(rhs) + 1e-2, (lhs, rhs)


def test_backward_image_halves_match(full):
    """ops.BACKWARD_PIPELINE (off by default): the backward in two image halves on two streams
    gives the single-launch gradients (d planes up to float-atomic order)."""
    from nfi import ops
    inp, meta = full
    a = _render(inp, meta, seed=3)
    old = ops.BACKWARD_PIPELINE
    ops.BACKWARD_PIPELINE = True
    try:
        b = _render(inp, meta, seed=3)
    finally:
        ops.BACKWARD_PIPELINE = old
    for k in ('d_palette', 'd_cam', 'd_focal'):
        assert torch.equal(a[k], b[k]), k
    assert rel_l2(b['d_planes'], a['d_planes']) < 1e-5


def _render_shapenet(inp, meta, sl, g_rgb, g_mask):
    """BASELINE configs[2]'s render: shapenet_chairs setting (scene_range 0.55, white background,
    camera not flipped), deterministic sampling, pose frozen (loaders.py:123 forces
    --inv_no_optimize_pose: force_no_cam_grad), gradients to planes and palette only."""
    nfi.configure(scene_range=0.55, white_background=True, fine_sampling=True)
    planes = inp['planes'][sl].to(DEV).requires_grad_()
    pal = inp['palette'][sl].to(DEV).requires_grad_()
    f = nfi.TriplaneField(planes=planes, palette=pal, w1=inp['w1'].to(DEV), b1=inp['b1'].to(DEV),
                          w2=inp['w2'].to(DEV), b2=inp['b2'].to(DEV), alpha=1.0, beta=0.1)
    rgb, depth, mask, _, _, _ = nfi.render(f, int(meta['H']), int(meta['W']), inp['cam'][sl].to(DEV),
                                           inp['focal'][sl].to(DEV), None, None, None, int(meta['S']),
                                           randomize=False, force_no_cam_grad=True)
    loss = (rgb * g_rgb[sl]).sum() + (mask * g_mask[sl]).sum()
    loss.backward()
    nfi.configure(white_background=False)
    return {'rgb': rgb.detach(), 'depth': depth.detach(), 'mask': mask.detach(), 'd_planes': planes.grad,
            'd_palette': pal.grad}


def test_shapenet_config_full_size():
    """configs[2] at full size (B=16, 128^2, 64+64, R=256): the batch render equals each image
    rendered alone (rays, samples and gradients are per image; the only batch coupling, the
    min/max near/far of missed rays, cannot change their zero weights): rgb / depth / mask and
    d palette bit for bit, d planes to summation order; repeat renders are deterministic; white-
    background bounds (rgb = sum w c + 1 - mask)."""
    B = 16
    inp, meta = synthetic_inputs(B=B, H=128, W=128, S=64, R=256, scene_range=0.55, seed=91,
                                 flipped=False, white_bg=True, randomize=False)
    g = torch.Generator().manual_seed(17)
    g_rgb = torch.randn(B, 128, 128, 3, generator=g).to(DEV)
    g_mask = torch.randn(B, 128, 128, generator=g).to(DEV)
    full = _render_shapenet(inp, meta, slice(0, B), g_rgb, g_mask)
    again = _render_shapenet(inp, meta, slice(0, B), g_rgb, g_mask)
    for k in ('rgb', 'depth', 'mask', 'd_palette'):
        assert torch.equal(full[k], again[k]), k
    assert rel_l2(full['d_planes'], again['d_planes']) < 1e-6
    m = full['mask']
    assert float(m.min()) >= 0.0 and float(m.max()) <= 1.0 + 1e-6
    assert 0.05 < float(m.mean()) < 0.95                       # neither empty nor opaque everywhere
    pal_max = float(inp['palette'].abs().max())
    bound = pal_max * m + (1 - m)
    assert bool((full['rgb'].abs() <= bound[..., None] * (1 + 1e-5) + 1e-6).all())
    assert float(full['depth'].min()) >= 0.0
    for k in (0, 7, 15):
        one = _render_shapenet(inp, meta, slice(k, k + 1), g_rgb, g_mask)
        for key in ('rgb', 'depth', 'mask', 'd_palette'):
            assert torch.equal(one[key][0], full[key][k]), (k, key)
        assert rel_l2(one['d_planes'][0], full['d_planes'][k]) < 1e-6, k


def _render_imagenet(inp, meta, sl, g_rgb, g_mask, randomize=False, seed=0):
    """BASELINE configs[4]'s per-GPU render (imagenet car 256², 128 coarse + 128 fine samples,
    pose gradients): the <SPL=2, NPL=4> kernel specialisation at full size."""
    nfi.configure(scene_range=float(meta['scene_range']), white_background=False, fine_sampling=True)
    planes = inp['planes'][sl].to(DEV).requires_grad_()
    pal = inp['palette'][sl].to(DEV).requires_grad_()
    cam = inp['cam'][sl].to(DEV).requires_grad_()
    focal = inp['focal'][sl].to(DEV).requires_grad_()
    f = nfi.TriplaneField(planes=planes, palette=pal, w1=inp['w1'].to(DEV), b1=inp['b1'].to(DEV),
                          w2=inp['w2'].to(DEV), b2=inp['b2'].to(DEV), alpha=1.0, beta=0.1)
    rgb, depth, mask, _, _, _ = nfi.render(f, int(meta['H']), int(meta['W']), cam, focal, None, None, None,
                                           int(meta['S']), randomize=randomize, seed=seed)
    loss = (rgb * g_rgb[sl]).sum() + (mask * g_mask[sl]).sum()
    loss.backward()
    return {'rgb': rgb.detach(), 'depth': depth.detach(), 'mask': mask.detach(), 'd_planes': planes.grad,
            'd_palette': pal.grad, 'd_cam': cam.grad, 'd_focal': focal.grad}


def test_imagenet_config_full_size():
    """configs[4]'s slice at full size (B=2, 256², 128+128, R=256, pose gradients): the batch render
    equals each image rendered alone (deterministic sampling: rgb / depth / mask / d palette bit for
    bit, d planes / d cam / d focal to float-atomic order); a randomized render repeats bit for bit
    with its seed and is bounded."""
    B, H = 2, 256
    inp, meta = synthetic_inputs(B=B, H=H, W=H, S=128, R=256, scene_range=1.4, seed=23)
    g = torch.Generator().manual_seed(29)
    g_rgb = torch.randn(B, H, H, 3, generator=g).to(DEV)
    g_mask = torch.randn(B, H, H, generator=g).to(DEV)
    full = _render_imagenet(inp, meta, slice(0, B), g_rgb, g_mask)
    for k in range(B):
        one = _render_imagenet(inp, meta, slice(k, k + 1), g_rgb, g_mask)
        for key in ('rgb', 'depth', 'mask', 'd_palette'):
            assert torch.equal(one[key][0], full[key][k]), (k, key)
        for key in ('d_planes', 'd_cam', 'd_focal'):
            assert rel_l2(one[key][0], full[key][k]) < 1e-5, (k, key)
    a = _render_imagenet(inp, meta, slice(0, B), g_rgb, g_mask, randomize=True, seed=8)
    b = _render_imagenet(inp, meta, slice(0, B), g_rgb, g_mask, randomize=True, seed=8)
    for key in ('rgb', 'depth', 'mask', 'd_palette'):
        assert torch.equal(a[key], b[key]), key
    m = a['mask']
    assert float(m.min()) >= 0.0 and float(m.max()) <= 1.0 + 1e-6 and float(m.mean()) > 0.05
    assert float(a['rgb'].abs().max()) <= float(inp['palette'].abs().max()) * (1 + 1e-6)
    assert float(a['depth'].min()) >= 0.0
