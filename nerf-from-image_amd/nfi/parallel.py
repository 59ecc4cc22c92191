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


def init_from_env(backend: str = 'nccl') -> Tuple[int, int, int]:
    """torchrun-style init (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*); returns (rank, local, world).
    Binds the process to its local GPU when backend is nccl (RCCL)."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if ws > 1 and not dist.is_initialized():
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
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return t.tolist()


def gather_rows(local: torch.Tensor, n_total: int) -> torch.Tensor:
    """Reassemble per-image results [n_local, ...] of every rank into [n_total, ...] in batch
    order (end-of-run report, run.py:2329-2404).  Ranks with empty chunks contribute nothing."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local
    ws = dist.get_world_size()
    bounds = chunk_bounds(n_total, ws)
    step = max(b - a for a, b in bounds)
    pad = torch.zeros((step,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:b - a] for p, (a, b) in zip(parts, bounds)], dim=0)
