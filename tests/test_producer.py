"""The caller side of the inversion step against the reference's own
outputs (tests/golden/producer.npz, pose.npz, inversion.npz; written by gen_golden.py from the
reference Generator, pose_utils and render() with the seeded weights of golden_io.load_seeded).

CPU: producer (mapping, synthesis, AttentionMapper) forward + latent gradient at full size — the
oracle's restatement of the reference op sequence over nfi.producer's modules
(oracle/producer_oracle.py; nfi's own producer runs on the GPU only: tests/test_gpu_inversion.py);
pose_to_matrix / matrix_to_pose; the inversion loop with the oracle as its renderer (the loop,
pose handling, Adam and producer are then the only things under test).
The GPU trajectory (HIP renderer in the loop) is tests/test_gpu_inversion.py.
"""

import json

import numpy as np
import pytest
import torch

from golden_io import load, load_seeded
from nfi import inversion, producer
from oracle.producer_oracle import ReferenceProducer


@pytest.fixture(scope='module')
def prod():
    d, meta = load('producer')
    gen = producer.InversionGenerator(scene_range=1.4)
    load_seeded(gen, int(meta['seed']))
    gen.requires_grad_(False)
    return ReferenceProducer(gen), d


def test_state_dict_matches_reference(prod):
    """A reference G_ema state_dict loads strictly: same keys, same shapes."""
    gen, d = prod
    ref_shapes = json.loads(d['sd_shapes'].item())
    ours = {k: list(v.shape) for k, v in gen.state_dict().items()}
    assert ours == ref_shapes


def test_mapping_network(prod):
    gen, d = prod
    w = gen.mapping_network(d['z'])
    assert w.shape == (2, 15, 512)
    torch.testing.assert_close(w, d['w_map'], rtol=1e-5, atol=1e-5)
    assert torch.equal(w[:, 0], w[:, 14])


def test_synthesis_and_palette(prod):
    gen, d = prod
    ws = d['ws'].clone().requires_grad_()
    planes, palette = gen.planes_and_palette(ws)
    assert planes.shape == (2, 3, 32, 256, 256)
    flat = planes.reshape(2, 96, 256, 256)
    tol = dict(rtol=1e-4, atol=1e-4 * float(d['planes_sample'].abs().max()))
    torch.testing.assert_close(flat.detach().reshape(-1)[d['idx']], d['planes_sample'], **tol)
    torch.testing.assert_close(flat.detach().double().sum(dim=(2, 3)), d['planes_chsum'],
                               rtol=1e-4, atol=1e-3 * float(d['planes_chabs'].max()) / 256)
    torch.testing.assert_close(flat.detach().double().abs().sum(dim=(2, 3)), d['planes_chabs'],
                               rtol=1e-5, atol=0)
    torch.testing.assert_close(palette.detach(), d['palette'], rtol=1e-5, atol=1e-6)
    seed = int(load('producer')[1]['seed'])
    gp = torch.randn(flat.shape, generator=torch.Generator().manual_seed(seed + 1))
    gq = torch.randn(palette.shape, generator=torch.Generator().manual_seed(seed + 2))
    ((flat * gp).sum() + (palette * gq).sum()).backward()
    scale = float(d['d_ws'].abs().max())
    torch.testing.assert_close(ws.grad, d['d_ws'], rtol=1e-3, atol=1e-4 * scale)


@pytest.mark.parametrize('name', ['pf', 'pu', 'of'])
def test_pose_roundtrip(name):
    d, _ = load('pose')
    flipped = name != 'pu'
    persp = f'{name}_z0' in d
    z0 = d[f'{name}_z0'] if persp else None
    mat, focal = inversion.pose_to_matrix(z0, d[f'{name}_t2'], d[f'{name}_s'], d[f'{name}_q'], flipped)
    torch.testing.assert_close(mat, d[f'{name}_mat'], rtol=1e-6, atol=1e-6)
    if persp:
        torch.testing.assert_close(focal, d[f'{name}_focal'], rtol=1e-6, atol=0)
    rz0, rt2, rs, rq = inversion.matrix_to_pose(d[f'{name}_mat'], d.get(f'{name}_focal'), flipped)
    torch.testing.assert_close(rt2, d[f'{name}_rt2'], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rs, d[f'{name}_rs'], rtol=1e-5, atol=0)
    torch.testing.assert_close(rq, d[f'{name}_rq'], rtol=1e-5, atol=1e-6)
    if persp:
        torch.testing.assert_close(rz0, d[f'{name}_rz0'], rtol=1e-5, atol=1e-6)
    # and the reference's own round trip: q recovered up to sign
    assert torch.allclose((rq * d[f'{name}_q']).sum(-1).abs(), torch.ones(rq.shape[0]), atol=1e-5)


def oracle_render_fn(scene_range):
    from oracle import render_oracle as orc

    def fn(gen, H, W, cam, focal, center, bbox, ws, S, force_no_cam_grad=False,
           u_coarse=None, u_fine=None):
        planes, palette = gen.planes_and_palette(ws)
        net = gen.decoder.net
        field = orc.Field(planes=planes, w1=net[0].weight, b1=net[0].bias, w2=net[2].weight,
                          b2=net[2].bias, palette=palette, alpha=gen.alpha, beta=gen.beta,
                          scene_range=scene_range)
        return orc.render(field, H, W, cam, focal, center, bbox, S, randomize=True,
                          force_no_cam_grad=force_no_cam_grad, u_coarse=u_coarse, u_fine=u_fine)
    return fn


def inversion_setup(device='cpu'):
    d, meta = load('inversion')
    gen = producer.InversionGenerator(scene_range=float(meta['scene_range']))
    load_seeded(gen, int(meta['seed']))
    with torch.no_grad():
        gen.decoder.net[2].bias[0] += float(meta['sdf_shift'])
    gen.requires_grad_(False).to(device)
    if str(device) == 'cpu':
        gen = ReferenceProducer(gen)      # the CPU loop: the reference's producer op sequence
    cfg = inversion.InversionConfig(steps=int(meta['steps']), resolution=int(meta['H']),
                                    samples=int(meta['S']), loss='l1',
                                    camera_flipped=bool(meta['flipped']))
    d = {k: v.to(device) for k, v in d.items()}
    return gen, d, meta, cfg


def check_trajectory(res, d, loss_rtol, w_rel):
    """Losses per step to `loss_rtol`; the latent by its distance to the reference's relative
    to how far the reference moved (`w_rel`), and by the share of coordinates off by a
    quarter of one Adam step or more (sign flips of gradients within rounding of zero: Adam's
    early steps move each coordinate by ~lr * gain * sign(grad)); pose parameters (gradients
    summed over whole images, far from zero) coordinate-wise, relative to how far each moved."""
    np.testing.assert_allclose(res.losses, d['losses'].cpu().numpy(), rtol=loss_rtol)
    ws, ref, w0 = res.ws.cpu(), d['ws'].cpu(), d['w_init'].cpu()
    moved = float((ref - w0).norm())
    assert moved > 0
    rel = float((ws - ref).norm()) / moved
    assert rel < w_rel, rel
    step = 2e-3 * 5.0
    flips = float(((ws - ref).abs() > 0.25 * step).float().mean())
    assert flips < 0.01, flips
    init = dict(zip(('z0', 't2', 's', 'q'),
                    inversion.matrix_to_pose(d['cam0'].cpu(), d['focal0'].cpu(), True)))
    for k in ('z0', 't2', 's', 'q'):
        ours, theirs = getattr(res, k).cpu(), d[k].cpu()
        moved_k = float((theirs - init[k]).abs().max())
        err = float((ours - theirs).abs().max())
        assert err <= w_rel * moved_k + 1e-7, (k, err, moved_k)
    return rel


def test_inversion_loop_with_oracle_renderer():
    gen, d, meta, cfg = inversion_setup()
    res = inversion.invert(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg,
                           uniforms=lambda it: (d['u_coarse'][it], d['u_fine'][it]),
                           render_fn=oracle_render_fn(float(meta['scene_range'])))
    check_trajectory(res, d, loss_rtol=1e-5, w_rel=1e-3)


def test_inversion_vgg_loss_needs_lpips_network():
    with pytest.raises(ValueError, match='LPIPS'):
        inversion.image_loss('vgg', torch.zeros(1, 2, 2, 3), torch.zeros(1, 2, 2, 3))
    with pytest.raises(NotImplementedError):
        inversion.image_loss('ssim', torch.zeros(1, 2, 2, 3), torch.zeros(1, 2, 2, 3))


@pytest.mark.parametrize('key', ['b', 'w'])
def test_augment_matches_reference(key):
    d, meta = load('augment')
    g = torch.Generator().manual_seed(int(meta[f'seed_{key}']))
    out = inversion.augment_images(d[f'{key}_img'], 1.0, white_background=key == 'w', generator=g)
    torch.testing.assert_close(out, d[f'{key}_out'], rtol=1e-6, atol=1e-6)


def test_inversion_default_renderer_is_hip_only():
    """Without render_fn the loop renders through nfi.render, which refuses CPU tensors."""
    gen, d, meta, cfg = inversion_setup()
    cfg.steps = 1
    with pytest.raises(RuntimeError, match='HIP devices only'):
        inversion.invert(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg,
                         uniforms=lambda it: (d['u_coarse'][it], d['u_fine'][it]))


def test_producer_refuses_cpu_tensors():
    """nfi's producer has one implementation, the HIP one: CPU tensors raise (no fallback)."""
    gen = producer.InversionGenerator(scene_range=1.4)
    gen.requires_grad_(False)
    with pytest.raises(RuntimeError, match='HIP devices only'):
        gen.planes_and_palette(torch.zeros(1, 15, 512))
    assert not hasattr(gen, 'set_backend')


def test_style_bank_layer_rows():
    """The style bank feeds every modulated layer the latent row SynthesisNetwork.forward gives it
    (block r gets rows[base : base + num_conv + 1]; conv0, conv1, toRGB in order)."""
    net = producer.SynthesisNetwork(512, 32, 96)
    rows = [k for _, k, _ in net._bank_layers()]
    # 4: conv1 0, rgb 1 | 8: conv0 1, conv1 2, rgb 3 | 16: 3, 4, 5 | 32: 5, 6, 7
    assert rows == [0, 1, 1, 2, 3, 3, 4, 5, 5, 6, 7]
    assert max(rows) + 1 == net.num_ws
