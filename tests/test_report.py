"""Inversion report / resume format and metrics (nfi/report.py).

Metrics pinned by tests/golden/metrics.npz (the reference's psnr / iou / rotation_matrix_distance);
the batch loop is exercised on the CPU with the oracle as its renderer (the HIP renderer is the
default; tests/test_gpu_inversion.py runs it on the GPU)."""

import torch

from golden_io import load
from nfi import inversion, report
from test_producer import inversion_setup, oracle_render_fn


def test_metrics_match_reference():
    d, _ = load('metrics')
    torch.testing.assert_close(report.psnr(d['pred'], d['tgt'], reduction='none'), d['psnr'],
                               rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(report.psnr(d['pred'], d['tgt']), d['psnr_mean'], rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(report.iou(d['a0'], d['a1'], reduction='none'), d['iou'])
    torch.testing.assert_close(report.rotation_matrix_distance(d['m0'], d['m1']), d['rot'],
                               rtol=1e-5, atol=1e-4)


def test_ssim_identities():
    g = torch.Generator().manual_seed(0)
    a = torch.rand(2, 3, 24, 24, generator=g)
    b = (a + 0.2 * torch.rand(2, 3, 24, 24, generator=g)).clamp(0, 1)
    s_same = report.ssim(a, a, reduction='none')
    torch.testing.assert_close(s_same, torch.ones(2), rtol=0, atol=1e-5)
    s = report.ssim(a, b, reduction='none')
    assert bool(((s > 0) & (s < 1)).all())
    torch.testing.assert_close(report.ssim(b, a, reduction='none'), s, rtol=1e-5, atol=1e-6)


def test_checkpoint_steps_rule():
    assert report.checkpoint_steps() == [0, 30]
    assert report.checkpoint_steps(gain_z=10) == [0, 10]
    assert report.checkpoint_steps(inv_steps=7) == [0, 7]
    assert report.checkpoint_steps(encoder_only=True) == [0]


def test_batch_loop_report_and_resume(tmp_path):
    gen, d, meta, cfg = inversion_setup()
    cfg.steps = 2
    n = 3
    images = torch.cat([d['target']] * 2)[:n]
    cams = torch.cat([d['cam0']] * 2)[:n]
    focals = torch.cat([d['focal0']] * 2)[:n]
    path = str(tmp_path / 'report_checkpoint.pth')
    lines = []
    rf = oracle_render_fn(float(meta['scene_range']))
    rep = report.run(gen, images, cams, focals, d['w_init'], cfg, test_bs=2, report_path=path,
                     log=lines.append, save_every=2, render_fn=rf, gt_cams=cams)
    assert sorted(rep) == [0, 2]
    for step in (0, 2):
        e = rep[step]
        assert e['ws'].shape == (n, 15, 512)
        for k in ('z0', 's', 'psnr', 'ssim', 'rot_error'):
            assert e[k].shape == (n,), k
        assert e['t2'].shape == (n, 2) and e['R'].shape == (n, 4)
        assert 'inception_activations_front' not in e          # empty keys dropped
    assert float(rep[0]['rot_error'].abs().max()) < 1e-2       # step 0 renders the given pose
    assert len(lines) == 2 and lines[0].startswith('[2/3] Finished batch in ') and lines[0].endswith(' s/img)')
    # the checkpoint written after the first batch resumes at image 2 with test_bs 2
    ck = report.load_checkpoint(path)
    assert ck is not None and ck[1] == 2 and ck[2] == 2
    assert len(ck[0][0]['ws']) == 1
    lines2 = []
    rep2 = report.run(gen, images, cams, focals, d['w_init'], cfg, test_bs=2, report_path=path,
                      log=lines2.append, save_every=2, render_fn=rf, gt_cams=cams)
    assert lines2 == [lines2[0]] and lines2[0].startswith('[3/3]')
    # images 0-1 come from the checkpoint; image 2 is re-inverted (fresh random draws)
    assert rep2[2]['ws'].shape == (n, 15, 512)
    assert torch.equal(rep2[2]['ws'][:2], rep[2]['ws'][:2])
    assert inversion.InversionConfig().steps == 30
