"""The inversion loop with the HIP renderer in it, against the reference's
trajectory (tests/golden/inversion.npz: run.py:1960-2310 around the reference Generator, render()
and pose_utils; 3 Adam steps, L1 loss, pose optimised, injected random draws).

The producer runs in PyTorch-ROCm on the GPU; the volume render (forward + backward to planes,
palette and the camera) is the HIP path.  Tolerances: losses to 1e-4 relative (the HIP render
matches the reference to fp32 rounding, tests/test_gpu_parity.py); latent and pose within 3%
of the distance the reference moved them (tests/test_producer.py::check_trajectory): the fp32
differences of the GPU producer (MIOpen; d_ws 4e-4 relative L2) and renderer in the gradient
feed Adam's normalised steps, where small gradient coordinates count as much as large ones
(measured 1.1-1.25%; the CPU oracle in the same loop stays below 0.1%).
"""

import pytest
import torch

import nfi
from nfi import inversion
from golden_io import load, load_seeded
from nfi import producer
from test_producer import check_trajectory, inversion_setup

pytestmark = pytest.mark.gpu


def test_inversion_trajectory_hip():
    dev = torch.device('cuda:0')
    gen, d, meta, cfg = inversion_setup(dev)
    nfi.configure(scene_range=float(meta['scene_range']), white_background=False,
                  fine_sampling=True, use_sdf=True, attention_values=10, use_viewdir=False)
    res = inversion.invert(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg,
                           uniforms=lambda it: (d['u_coarse'][it], d['u_fine'][it]))
    rel = check_trajectory(res, d, loss_rtol=1e-4, w_rel=3e-2)
    print(f'latent distance / reference displacement: {rel:.2e}')


def test_inversion_decreases_loss_hip():
    """30 steps at 64² (Philox draws): the L1 loss goes down and the pose stays valid."""
    dev = torch.device('cuda:0')
    gen, d, meta, cfg = inversion_setup(dev)
    nfi.configure(scene_range=float(meta['scene_range']), white_background=False)
    cfg.steps, cfg.resolution, cfg.samples = 30, 64, 32
    target = torch.nn.functional.interpolate(d['target'].permute(0, 3, 1, 2), size=(64, 64),
                                             mode='bilinear', align_corners=False).permute(0, 2, 3, 1)
    res = inversion.invert(gen, target.contiguous(), d['cam0'], d['focal0'], d['w_init'], cfg)
    assert len(res.losses) == 30
    assert min(res.losses[-5:]) < res.losses[0]
    assert torch.allclose(res.q.norm(dim=-1), torch.ones(res.q.shape[0], device=dev), atol=1e-5)
    assert bool((res.s > 0).all()) and bool((res.z0.abs() <= 4).all())


def test_producer_on_gpu():
    """The producer on the GPU (MIOpen convolutions) against the reference's CPU outputs."""
    dev = torch.device('cuda:0')
    d, meta = load('producer')
    gen = producer.InversionGenerator(scene_range=1.4)           # backend 'hip'
    load_seeded(gen, int(meta['seed']))
    gen.requires_grad_(False).to(dev)
    ws = d['ws'].to(dev).requires_grad_()
    planes, palette = gen.planes_and_palette(ws)
    flat = planes.reshape(2, 96, 256, 256)
    sample = flat.detach().reshape(-1)[d['idx'].to(dev)].cpu()
    scale = float(d['planes_sample'].abs().max())
    err = float((sample - d['planes_sample']).abs().max()) / scale
    seed = int(meta['seed'])
    gp = torch.randn(flat.shape, generator=torch.Generator().manual_seed(seed + 1)).to(dev)
    gq = torch.randn(palette.shape, generator=torch.Generator().manual_seed(seed + 2)).to(dev)
    ((flat * gp).sum() + (palette * gq).sum()).backward()
    g = ws.grad.cpu()
    gerr = float((g - d['d_ws']).norm() / d['d_ws'].norm())
    print(f'producer on GPU: planes max err / max {err:.2e}, d_ws rel L2 err {gerr:.2e}')
    assert err < 1e-4
    torch.testing.assert_close(palette.detach().cpu(), d['palette'], rtol=1e-4, atol=1e-5)
    assert gerr < 1e-3


def test_report_batch_loop_hip(tmp_path):
    """nfi.report.run with the HIP renderer and producer: report layout and s/img lines."""
    from nfi import lpips, report
    dev = torch.device('cuda:0')
    gen, d, meta, cfg = inversion_setup(dev)
    nfi.configure(scene_range=float(meta['scene_range']), white_background=False)
    cfg.steps = 3
    lines = []
    rep = report.run(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg, test_bs=2,
                     report_path=str(tmp_path / 'ck.pth'), lpips_net=lpips.LPIPS().to(dev),
                     gt_cams=d['cam0'], log=lines.append)
    assert sorted(rep) == [0, 3] and len(lines) == 1
    for k in ('ws', 'psnr', 'ssim', 'lpips', 'rot_error'):
        assert rep[3][k].shape[0] == 2, k
    assert torch.isfinite(rep[3]['psnr']).all()
