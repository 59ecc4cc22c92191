"""The inversion step's folded small ops against their torch formulations in fp64: the pose algebra
(nfi_pose_forward / _backward / _project: pose_to_matrix(z0, t2, s, F.normalize(q)) of
lib/pose_utils.py:48-78 and the post-step projections of run.py:2300-2306) and the AttentionMapper's
conditional norm + activation (nfi_syn_cond_norm_act_*: generator.py:42-60, 173-178) — forward
values and gradients."""

import pytest
import torch
import torch.nn.functional as F

from nfi import inversion, producer_ops

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g, dtype=torch.float64) * scale


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


@pytest.mark.parametrize('with_z0', [True, False])
@pytest.mark.parametrize('flipped', [True, False])
@pytest.mark.parametrize('B', [1, 4, 70])
def test_pose_matrix_matches_torch(with_z0, flipped, B):
    z0 = _rand(B, seed=1, scale=0.5) if with_z0 else None
    t2 = _rand(B, 2, seed=2, scale=0.3)
    s = _rand(B, seed=3).abs() + 0.5
    q = _rand(B, 4, seed=4) * 1.7          # not unit: the normalisation is part of the op
    g_cam = _rand(B, 4, 4, seed=5)
    g_f = _rand(B, seed=6) if with_z0 else None

    def run(dev, dtype, fn):
        ins = [None if t is None else t.detach().to(dev, dtype).clone().requires_grad_() for t in (z0, t2, s, q)]
        cam, foc = fn(*ins)
        loss = (cam * g_cam.to(dev, dtype)).sum()
        if foc is not None:
            loss = loss + (foc * g_f.to(dev, dtype)).sum()
        loss.backward()
        return cam, foc, [None if t is None else t.grad for t in ins]

    ref = run('cpu', torch.float64,
              lambda a, b, c, d: inversion.pose_to_matrix(a, b, c, F.normalize(d, dim=-1), flipped))
    hip = run(DEV, torch.float32, lambda a, b, c, d: inversion.pose_matrix(a, b, c, d, flipped))
    assert _rel(hip[0], ref[0]) < 2e-6
    if with_z0:
        assert _rel(hip[1], ref[1]) < 2e-6
    else:
        assert hip[1] is None and ref[1] is None
    for gh, gr in zip(hip[2], ref[2]):
        if gr is None:
            assert gh is None
        else:
            assert _rel(gh, gr) < 1e-5, (gh, gr)


def test_pose_project_matches_torch():
    B = 6
    z0 = (_rand(B, seed=7) * 5).float()
    s = _rand(B, seed=8).float()
    q = (_rand(B, 4, seed=9) * 3).float()
    zr, sr, qr = z0.clone(), s.clone(), q.clone()
    inversion.project_pose(zr, sr, qr)          # the CPU (torch) form
    zd, sd, qd = z0.to(DEV), s.to(DEV), q.to(DEV)
    inversion.project_pose(zd, sd, qd)
    torch.testing.assert_close(zd.cpu(), zr, rtol=0, atol=0)
    torch.testing.assert_close(sd.cpu(), sr, rtol=0, atol=0)
    torch.testing.assert_close(qd.cpu(), qr, rtol=2e-7, atol=1e-7)
    inversion.project_pose(None, sd, qd)        # no focal parameter
    torch.testing.assert_close(sd.cpu(), sr, rtol=0, atol=0)


@pytest.mark.parametrize('B,C,strided', [(4, 512, True), (3, 512, False), (2, 100, True), (1, 1024, False)])
def test_cond_norm_act_matches_torch(B, C, strided):
    h = _rand(B, C, seed=10) * 3 + 0.5
    if strided:                                 # gamma1 / beta as views of one [B, 8C] projection
        proj = _rand(B, 8 * C, seed=11)
        proj[:, :C] += 1.0
        g1, be = proj[:, :C], proj[:, C:2 * C]
    else:
        g1, be = _rand(B, C, seed=12) + 1.0, _rand(B, C, seed=13)
    gx = _rand(B, C, seed=14)

    def run(dev, dtype, fn):
        if strided:
            p = proj.detach().to(dev, dtype).clone().requires_grad_()
            a, b = p[:, :C], p[:, C:2 * C]
            leaves = [p]
        else:
            a, b = g1.detach().to(dev, dtype).clone().requires_grad_(), be.detach().to(dev, dtype).clone().requires_grad_()
            leaves = [a, b]
        hh = h.detach().to(dev, dtype).clone().requires_grad_()
        x = fn(hh, a, b)
        (x * gx.to(dev, dtype)).sum().backward()
        return x, [hh.grad] + [t.grad for t in leaves]

    ref = run('cpu', torch.float64, lambda hh, a, b: F.leaky_relu(torch.addcmul(b, a, F.layer_norm(hh, (C,))), 0.2))
    hip = run(DEV, torch.float32, producer_ops.cond_norm_act)
    assert _rel(hip[0], ref[0]) < 2e-6
    for gh, gr in zip(hip[1], ref[1]):
        assert _rel(gh, gr) < 1e-5
