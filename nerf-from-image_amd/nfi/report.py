"""Inversion report / resume format and the s/img harness:
run.py:1820-1850 (checkpoint steps, report layout), 2020-2110 (evaluate_inversion), 2319-2336
(per-batch s/img line, report checkpoint every 512 images), 2340-2404 (consolidation, report.pth).

The report is `{step: {key: [per-batch CPU tensors]}}` with the reference's keys; checkpoints are
`{'report', 'idx', 'test_bs'}` written with torch.save and read back with
torch.load(weights_only=True) (plain tensors, lists, dicts and ints only), so a report written
here resumes in the reference and vice versa.

Metrics (lib/metrics.py, lib/pose_utils.py): psnr, iou, rotation_matrix_distance restated; ssim
restates scikit-image's `structural_similarity` defaults (7x7 uniform window, sample
covariance, K1 0.01, K2 0.03, data_range 1, per-channel mean) on scipy.ndimage.uniform_filter —
the filter scikit-image itself uses — since scikit-image is not in this image (parity of ssim
unpinned).  Inception/FID activations are outside the path (their keys stay empty and are
dropped by `consolidate`, as the reference drops empty keys).
"""

from __future__ import annotations

import math
import os
from typing import Iterable, Optional

import numpy as np
import torch
import torch.nn.functional as F

REPORT_KEYS = ('ws', 'z0', 'R', 's', 't2', 'psnr', 'psnr_random', 'lpips', 'lpips_random', 'ssim',
               'ssim_random', 'iou', 'rot_error', 'inception_activations_front',
               'inception_activations_random')


def checkpoint_steps(inv_steps: Optional[int] = None, gain_z: float = 5,
                     encoder_only: bool = False) -> list:
    """run.py:1822-1830."""
    if encoder_only:
        return [0]
    if inv_steps:
        return [0, inv_steps]
    if gain_z >= 10:
        return [0, 10]
    return [0, 30]


def new_report(steps: Iterable[int]) -> dict:
    return {step: {k: [] for k in REPORT_KEYS} for step in steps}


def save_checkpoint(path: str, report: dict, idx: int, test_bs: int):
    """run.py:2329-2336 (written every 512 images)."""
    tmp = path + '.tmp'
    with open(tmp, 'wb') as f:
        torch.save({'report': report, 'idx': idx, 'test_bs': test_bs}, f)
    os.replace(tmp, path)


def load_checkpoint(path: str):
    """run.py:1858-1870 -> (report, idx, test_bs), or None if absent."""
    if not os.path.exists(path):
        return None
    with open(path, 'rb') as f:
        ck = torch.load(f, weights_only=True)
    return ck['report'], int(ck['idx']), int(ck['test_bs'])


def consolidate(report: dict) -> dict:
    """run.py:2340-2347: concatenate per-batch lists, drop empty keys (in place)."""
    for entry in report.values():
        for k, v in list(entry.items()):
            if len(v) == 0:
                del entry[k]
            else:
                entry[k] = torch.cat(v, dim=0)
    return report


def batch_line(idx: int, total: int, seconds: float, test_bs: int) -> str:
    """run.py:2319-2323."""
    return f'[{idx}/{total}] Finished batch in {seconds} s ({seconds / test_bs} s/img)'


# ---------------------------------------------------------------------------------------------
# metrics

def _range_check(im):
    eps = 1e-1
    if not (float(im.max()) < 1 + eps and float(im.min()) > -eps):
        raise AssertionError('Range check failed')


def psnr(pred, target, reduction='mean'):
    """metrics.py:30-55 (no mask): images in [0,1], [b,3,H,W] or [b,H,W,3]; clamp at 60 dB."""
    assert pred.shape == target.shape and pred.dim() == 4
    _range_check(pred)
    _range_check(target)
    pred, target = pred.clamp(0, 1), target.clamp(0, 1)
    v = (-10 * torch.log10((pred - target).square().mean(dim=[1, 2, 3]))).clamp(max=60)
    return v.mean() if reduction == 'mean' else v


def iou(alpha_pred, alpha_real, reduction='mean'):
    """metrics.py:88-103."""
    assert alpha_pred.shape == alpha_real.shape
    _range_check(alpha_pred)
    _range_check(alpha_real)
    a, b = alpha_pred > 0.5, alpha_real > 0.5
    inter = (a & b).float().sum(dim=[-2, -1])
    union = (a | b).float().sum(dim=[-2, -1])
    v = (inter + 1e-6) / (union + 1e-6)
    return v.mean() if reduction == 'mean' else v.flatten()


def rotation_matrix_distance(p, q):
    """pose_utils.py:160-168: geodesic distance in degrees."""
    if p.shape[-1] == 4:
        p = p[:, :3, :3] / p[:, 3:4, 3:4]
        q = q[:, :3, :3] / q[:, 3:4, 3:4]
    pqt = p @ q.transpose(-2, -1)
    trace = pqt[:, 0, 0] + pqt[:, 1, 1] + pqt[:, 2, 2]
    return torch.acos(((trace - 1) / 2).clamp(-1, 1)) / math.pi * 180


def _ssim_channel(x: np.ndarray, y: np.ndarray, win: int = 7) -> float:
    from scipy.ndimage import uniform_filter
    npix = win * win
    cov_norm = npix / (npix - 1)
    ux, uy = uniform_filter(x, size=win), uniform_filter(y, size=win)
    uxx, uyy, uxy = uniform_filter(x * x, size=win), uniform_filter(y * y, size=win), uniform_filter(x * y, size=win)
    vx, vy, vxy = cov_norm * (uxx - ux * ux), cov_norm * (uyy - uy * uy), cov_norm * (uxy - ux * uy)
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    s = ((2 * ux * uy + c1) * (2 * vxy + c2)) / ((ux * ux + uy * uy + c1) * (vx + vy + c2))
    pad = (win - 1) // 2
    return float(s[pad:-pad, pad:-pad].astype(np.float64).mean())


def ssim(pred, target, reduction='mean'):
    """metrics.py:58-85: [b,3,H,W] in [0,1]; scikit-image structural_similarity per image
    (channel_axis=0, data_range=1), or over the flattened batch for reduction='mean'."""
    assert pred.shape == target.shape and pred.dim() == 4 and pred.shape[1] == 3
    _range_check(pred)
    _range_check(target)
    p = pred.clamp(0, 1).detach().cpu().numpy()
    t = target.clamp(0, 1).detach().cpu().numpy()
    if reduction == 'mean':
        p, t = p.reshape(-1, *p.shape[2:]), t.reshape(-1, *t.shape[2:])
        return torch.tensor([np.mean([_ssim_channel(a, b) for a, b in zip(p, t)])], dtype=torch.float32)
    return torch.tensor([np.mean([_ssim_channel(a, b) for a, b in zip(pe, te)]) for pe, te in zip(p, t)],
                        dtype=torch.float32)


# ---------------------------------------------------------------------------------------------
# evaluate_inversion (run.py:2020-2110, the front view)

@torch.no_grad()
def evaluate(report: dict, it: int, generator, params, target_img, resolution: int, samples: int,
             camera_flipped: bool, center=None, bbox=None, gain_z: float = 5.0, lpips_net=None,
             gt_cam2world=None, has_mask: bool = False, render_fn=None):
    """Render the current estimate (no pose gradient) and append ws, pose and the metrics to
    report[it].  `params` = (z_, z0_, t2_, s_, q_) as held by the optimiser; `target_img`
    [b,H,W,3 or 4] in [-1,1] (4th channel: mask)."""
    from .inversion import pose_to_matrix
    from .render import render
    z_, z0_, t2_, s_, q_ = params
    item = report[it]

    def snap(t):
        # a copy even on the host (.cpu() of a CPU tensor is the live parameter Adam keeps updating)
        return t.detach().to('cpu', copy=True)
    ws = z_.detach() * gain_z
    item['ws'].append(snap(ws))
    if z0_ is not None:
        item['z0'].append(snap(z0_))
    item['R'].append(snap(q_))
    item['s'].append(snap(s_))
    item['t2'].append(snap(t2_))
    cam, focal = pose_to_matrix(None if z0_ is None else z0_.detach(), t2_.detach(), s_.detach(),
                                F.normalize(q_.detach(), dim=-1), camera_flipped)
    if ws.shape[1] == 1:
        ws = ws.expand(-1, 15, -1)
    out = (render_fn or render)(generator, resolution, resolution, cam, focal, center, bbox, ws,
                                samples, force_no_cam_grad=True)
    rgb, acc = out[0], out[2]
    pred = rgb.permute(0, 3, 1, 2).clamp(-1, 1)
    tgt = target_img.permute(0, 3, 1, 2)
    item['psnr'].append(psnr(pred[:, :3] / 2 + 0.5, tgt[:, :3] / 2 + 0.5, reduction='none').cpu())
    item['ssim'].append(ssim(pred[:, :3] / 2 + 0.5, tgt[:, :3] / 2 + 0.5, reduction='none').cpu())
    if has_mask and tgt.shape[1] > 3:
        item['iou'].append(iou(acc, tgt[:, 3], reduction='none').cpu())
    if lpips_net is not None:
        item['lpips'].append(lpips_net(pred[:, :3], tgt[:, :3]).flatten().cpu())
    if gt_cam2world is not None:
        item['rot_error'].append(rotation_matrix_distance(cam, gt_cam2world).cpu())
    return rgb


def _gather_report_rows(report: dict, it: int, local: dict):
    """Append to report[it] the per-image rows every rank recorded for its chunk of the batch,
    in rank (= batch) order.  The rows are a few KB per image of CPU tensors (ws is the largest,
    30 KB), so they travel as objects; ranks with an empty chunk send nothing."""
    import torch.distributed as dist
    rows = {k: torch.cat(v, dim=0) for k, v in local.items() if len(v)}
    every = [None] * dist.get_world_size()
    dist.all_gather_object(every, rows)
    for k in REPORT_KEYS:
        parts = [r[k] for r in every if k in r]
        if parts:
            report[it][k].append(torch.cat(parts, dim=0))


def run(generator, images, cams, focals, w_init, cfg, test_bs: int, report_path: str,
        steps: Optional[list] = None, lpips_net=None, gt_cams=None, has_mask: bool = False,
        log=print, save_every: int = 512, render_fn=None, uniforms=None, distributed: Optional[bool] = None):
    """The batch loop of run.py:1872-2336 over a set of target images: resume from
    `report_path` (report_checkpoint.pth) if present, invert `test_bs` images at a time
    (falling back to 1 for a short tail, run.py:1879), evaluate at the checkpoint steps, log the
    s/img line, checkpoint every `save_every` images.  Returns the consolidated report.

    Under torch.distributed (`distributed` None = whenever a process group of >1 ranks exists)
    `test_bs` is the GLOBAL batch, as the reference's `batch_size // 4 * len(gpu_ids)`
    (run.py:1757): every rank calls run() with the same arguments, each batch is split over the
    ranks by nfi.parallel.invert_sharded (DataParallel's torch.chunk), each rank evaluates its own
    images, and the per-image report rows are gathered in batch order, so every rank returns the
    same report as one process inverting the whole batch.  Rank 0 alone logs and writes the
    report checkpoint.  `uniforms(idx, it) -> (u_coarse, u_fine)` injects the renderer's draws
    of batch `idx` (tests)."""
    import time as _time
    from .inversion import invert
    from .parallel import invert_sharded, world
    rank, ws = world()
    sharded = ws > 1 if distributed is None else distributed
    steps = steps or checkpoint_steps(cfg.steps, cfg.gain_z)
    cfg.steps = max(steps)
    report, idx = new_report(steps), 0
    ck = load_checkpoint(report_path)
    if ck is not None:
        report, idx, test_bs = ck
    n = images.shape[0]
    while idx < n:
        t1 = _time.time()
        if test_bs != 1 and images[idx:idx + test_bs].shape[0] < test_bs:
            test_bs = 1
        sl = slice(idx, idx + test_bs)
        tgt = images[sl]
        gt = None if gt_cams is None else gt_cams[sl]
        unif = None if uniforms is None else (lambda it, i0=idx: uniforms(i0, it))

        def on_checkpoint(it, params, tgt=tgt, gt=gt, chunk=None):
            if chunk is None:
                evaluate(report, it, generator, params, tgt, cfg.resolution, cfg.samples,
                         cfg.camera_flipped, gain_z=cfg.gain_z, lpips_net=lpips_net,
                         gt_cam2world=gt, has_mask=has_mask, render_fn=render_fn)
                return
            a, e = chunk
            local = new_report([it])
            if params is not None:
                evaluate(local, it, generator, params, tgt[a:e], cfg.resolution, cfg.samples,
                         cfg.camera_flipped, gain_z=cfg.gain_z, lpips_net=lpips_net,
                         gt_cam2world=None if gt is None else gt[a:e], has_mask=has_mask, render_fn=render_fn)
            _gather_report_rows(report, it, local[it])

        foc = None if focals is None else focals[sl]
        if sharded:
            invert_sharded(generator, tgt, cams[sl], foc, w_init, cfg, uniforms=unif, lpips_net=lpips_net,
                           render_fn=render_fn, checkpoints=steps, on_checkpoint=on_checkpoint)
        else:
            invert(generator, tgt, cams[sl], foc, w_init, cfg, uniforms=unif, lpips_net=lpips_net,
                   checkpoints=steps, on_checkpoint=on_checkpoint, render_fn=render_fn)
        idx += test_bs
        if rank == 0:
            log(batch_line(idx, n, _time.time() - t1, test_bs))
            if idx % save_every == 0:
                save_checkpoint(report_path, report, idx, test_bs)
    return consolidate(report)
