"""Seeded synthetic inversion inputs at the real sizes for bench.py and the
multi-GPU harness: no datasets or checkpoints exist offline, so planes are N(0, 1.87^2)
(the measured std of the random-init synthesis output), the decoder is a random
EqualizedLinear init with the -0.97 SDF bias shift, the palette is
wide_sigmoid_rescaled(N(0,1)), and cameras sit on a sphere of radius 3.3*scene_range with
focal 1.859 (pose_utils.pose_to_matrix convention)."""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .inversion import pose_to_matrix
from .render import TriplaneField


def inversion_batch(B, H, W, S, R, scene_range, seed, flipped=True, device='cuda', texel_major=False):
    """texel_major: the planes [B,3,32,R,R] held in [B,3,R,R,32] storage (same values) — the layout
    InversionGenerator's 'hip' backend emits and the renderer reads with no conversion pass."""
    g = torch.Generator(device=device).manual_seed(seed)
    dev = torch.device(device)
    planes = 1.87 * torch.randn((B, 3, 32, R, R), generator=g, device=dev)
    if texel_major:
        planes = planes.permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)
    w1 = torch.randn((64, 32), generator=g, device=dev)
    w2 = torch.randn((11, 64), generator=g, device=dev)
    b1 = torch.zeros(64, device=dev)
    b2 = torch.zeros(11, device=dev)
    b2[0] -= 0.97
    palette = torch.sigmoid(torch.randn((B, 10, 3), generator=g, device=dev)) * 2.004 - 1.002
    q = F.normalize(torch.randn((B, 4), generator=g, device=dev), dim=-1)
    t2 = 0.05 * torch.randn((B, 2), generator=g, device=dev)
    f = 2 * 1.859
    s = torch.full((B,), f / (3.3 * scene_range), device=dev)
    z0 = torch.full((B,), math.log(f - 1), device=dev)
    cam, focal = pose_to_matrix(z0, t2, s, q, flipped)
    field = TriplaneField(planes=planes.requires_grad_(), palette=palette.requires_grad_(),
                          w1=w1, b1=b1, w2=w2, b2=b2, alpha=1.0, beta=0.1)
    return {'field': field, 'cam': cam, 'focal': focal,
            'g_rgb': torch.randn((B, H, W, 3), generator=g, device=dev),
            'g_mask': torch.randn((B, H, W), generator=g, device=dev)}


def cameras(B, scene_range, seed, flipped=True, device='cuda'):
    """B seeded cameras of inversion_batch's distribution (random unit quaternion, small t2,
    focal 1.859 at 3.3*scene_range) from their own stream: every rank of a sharded run draws the
    same whole-batch cameras -> (cam2world [B,4,4], focal [B])."""
    g = torch.Generator(device=device).manual_seed(seed)
    dev = torch.device(device)
    q = F.normalize(torch.randn((B, 4), generator=g, device=dev), dim=-1)
    t2 = 0.05 * torch.randn((B, 2), generator=g, device=dev)
    f = 2 * 1.859
    s = torch.full((B,), f / (3.3 * scene_range), device=dev)
    z0 = torch.full((B,), math.log(f - 1), device=dev)
    return pose_to_matrix(z0, t2, s, q, flipped)
