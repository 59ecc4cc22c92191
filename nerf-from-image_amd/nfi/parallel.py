"""One process per GPU for the inversion renderer (replaces the reference's single-process
`nn.DataParallel(ParallelModel(...))`, run.py:636-640).

The inversion batch is embarrassingly parallel: each image's latent, pose and
Adam state are private, the generator is frozen, and the loss is a sum of per-image terms, so
no gradient is ever reduced.  Each rank therefore renders and optimises its own contiguous
chunk of the step batch — `torch.chunk` semantics, exactly what DataParallel's Scatter gives
each replica (ceil(b/n) per rank) — with no collective on the data path.  Collectives are
only used off the hot path: an optional sum of logging scalars per step and one all_gather of
per-image results at the end (RCCL over xGMI under backend "nccl"; gloo on CPU for tests).
"""

from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    """(rank, world_size) of the default process group, (0, 1) when not distributed."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


# Test-only switch: run the collectives of gather_rows / sum_across / invert_sharded even in a
# 1-rank group (they return early at world size 1), so a single-GPU box executes the RCCL branch
# (tests/test_gpu_rccl.py).  Never set by the product.
FORCE_COLLECTIVES = False


def _collective() -> bool:
    """True when a collective must run: a group of > 1 ranks, or any group under FORCE_COLLECTIVES."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or FORCE_COLLECTIVES


def init_from_env(backend: str = 'nccl', force: bool = False) -> Tuple[int, int, int]:
    """torchrun-style init (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*); returns (rank, local, world).
    Binds the process to its local GPU when backend is nccl (RCCL).  A 1-rank world creates no
    group unless `force` (the RCCL test on a one-GPU box)."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if (ws > 1 or force) and not dist.is_initialized():
        if backend == 'nccl':
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    return rank, local, ws


def chunk_bounds(n: int, world_size: int) -> List[Tuple[int, int]]:
    """[start, stop) of each rank's chunk with torch.chunk semantics: ceil(n/world) items per
    chunk, trailing ranks may get fewer or none (DataParallel Scatter, run.py:636)."""
    if n <= 0:
        return [(0, 0)] * world_size
    step = -(-n // world_size)
    out = []
    for r in range(world_size):
        a = min(n, r * step)
        out.append((a, min(n, a + step)))
    return out


def shard(tensors: Dict[str, torch.Tensor], rank: int, world_size: int) -> Dict[str, torch.Tensor]:
    """This rank's slice (along dim 0) of every per-image tensor of the step batch."""
    n = {v.shape[0] for v in tensors.values()}
    if len(n) != 1:
        raise ValueError(f'inconsistent batch sizes {n}')
    a, b = chunk_bounds(n.pop(), world_size)[rank]
    return {k: v[a:b] for k, v in tensors.items()}


def sum_scalars(values: Sequence[float], device) -> List[float]:
    """Optional per-step logging reduction (loss, sum psnr, sum lpips): one all_reduce."""
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if _collective():
        dist.all_reduce(t)
    return t.tolist()


def _comm_device(t: torch.Tensor) -> torch.device:
    """Where a collective's buffer must live: the rank's GPU under RCCL ('nccl'), the host under gloo."""
    if dist.get_backend() == 'nccl':
        return torch.device('cuda', torch.cuda.current_device())
    return torch.device('cpu')


def gather_rows(local: torch.Tensor, n_total: int) -> torch.Tensor:
    """Reassemble per-image results [n_local, ...] of every rank into [n_total, ...] in batch
    order (end-of-run report, run.py:2329-2404).  Ranks with empty chunks contribute nothing.
    The result is on `local`'s device (the collective itself runs where the backend needs it)."""
    if not _collective():
        return local
    ws = dist.get_world_size()
    bounds = chunk_bounds(n_total, ws)
    if local.shape[0] != (lambda ab: ab[1] - ab[0])(bounds[dist.get_rank()]):
        raise ValueError(f'rank {dist.get_rank()} holds {local.shape[0]} rows, its chunk of {n_total} '
                         f'is {bounds[dist.get_rank()]}')
    step = max(b - a for a, b in bounds)
    cdev = _comm_device(local)
    pad = torch.zeros((step,) + tuple(local.shape[1:]), dtype=local.dtype, device=cdev)
    pad[:local.shape[0]] = local.detach().to(cdev)
    parts = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:b - a] for p, (a, b) in zip(parts, bounds)], dim=0).to(local.device)


def sum_across(values: torch.Tensor) -> torch.Tensor:
    """all_reduce(SUM) of a small tensor (per-step logging terms), returned on its own device."""
    if not _collective():
        return values
    t = values.detach().to(_comm_device(values), torch.float64).clone()
    dist.all_reduce(t)
    return t.to(values.device, values.dtype)


def invert_sharded(generator, target_img: torch.Tensor, cam2world: torch.Tensor, focal, w_init: torch.Tensor,
                   cfg, center=None, bbox=None, uniforms=None, lpips_net=None, render_fn=None,
                   checkpoints=(), on_checkpoint=None):
    """The inversion of one step batch split over the ranks (run.py:1757: the batch is
    `batch_size // 4 * len(gpu_ids)` images and DataParallel hands each GPU a torch.chunk of
    it, run.py:636-640, 2264-2282).  Every rank passes the WHOLE batch (targets, cameras,
    focals, per-image latents); this rank inverts rows chunk_bounds(b, world)[rank] with
    nfi.inversion.invert (its own latent, pose and Adam state — nothing is shared, so no
    gradient is reduced), and the per-image results are all_gathered back into batch order:
    every rank returns the InversionResult of the whole batch.  `losses` are the per-step loss
    sums over all images (one all_reduce at the end, not per step).

    `uniforms(it) -> (u_coarse, u_fine)` of the whole batch ([b*H*W*S] each, image-major) is
    sliced to this rank's images, so a sharded run with injected draws reproduces the unsharded
    one image for image.  `on_checkpoint(it, params)` sees this rank's chunk of the parameters
    and `chunk` = (start, stop) as a keyword (nfi.report.run gathers what it records)."""
    from .inversion import InversionResult, invert
    rank, ws = world()
    b = target_img.shape[0]
    a, e = chunk_bounds(b, ws)[rank]

    def rows(t):
        if t is None or not torch.is_tensor(t) or t.dim() == 0 or t.shape[0] != b:
            return t
        return t[a:e]

    loc_uniforms = None
    if uniforms is not None:
        def loc_uniforms(it):
            out = []
            for u in uniforms(it):
                if u is not None:
                    if u.shape[0] % b:
                        raise ValueError(f'draws of shape {tuple(u.shape)} are not image-major over {b} images')
                    per = u.shape[0] // b                # leading rows per image ([b,...], [b*HW,S], [b*HW*S])
                    u = u[a * per:e * per]
                out.append(u)
            return tuple(out)

    loc_ckpt = None
    if on_checkpoint is not None:
        def loc_ckpt(it, params):
            on_checkpoint(it, params, chunk=(a, e))

    dev = target_img.device
    if e > a:
        w_loc = w_init if w_init.shape[0] != b else w_init[a:e]
        res = invert(generator, target_img[a:e], cam2world[a:e], rows(focal), w_loc, cfg, center=rows(center),
                     bbox=rows(bbox), uniforms=loc_uniforms, render_fn=render_fn, lpips_net=lpips_net,
                     checkpoints=checkpoints, on_checkpoint=loc_ckpt)
        losses = torch.tensor(res.losses, dtype=torch.float64, device=dev)
        parts = res
    else:
        # an empty chunk (b < world): nothing to invert; still joins every collective, in the order
        # invert() fires them on the other ranks: each step in [0, cfg.steps] once, ascending
        if on_checkpoint is not None:
            for it in sorted({int(c) for c in checkpoints if 0 <= int(c) <= cfg.steps}):
                on_checkpoint(it, None, chunk=(a, e))
        losses = torch.zeros(cfg.steps, dtype=torch.float64, device=dev)
        parts = None
    total = sum_across(losses)

    def gathered(name, like_shape):
        if parts is not None:
            loc = getattr(parts, name)
        else:
            loc = torch.zeros((0,) + like_shape, device=dev)
        return gather_rows(loc, b) if (ws > 1 or FORCE_COLLECTIVES) else loc

    ws_all = gathered('ws', (15, w_init.shape[-1]))
    z0_all = None if focal is None else gathered('z0', ())
    t2_all = gathered('t2', (2,))
    s_all = gathered('s', ())
    q_all = gathered('q', (4,))
    return InversionResult(ws=ws_all, z0=z0_all, t2=t2_all, s=s_all, q=q_all,
                           losses=[float(x) for x in total.tolist()],
                           seconds=0.0 if parts is None else parts.seconds)
