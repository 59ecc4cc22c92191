"""Multi-process (world_size 2, gloo on CPU) coverage of the one-process-per-GPU path: the
step batch is split with DataParallel's torch.chunk semantics, every rank renders its own
images (CPU oracle stands in for the HIP renderer here — no GPU), and the end-of-run gather
reassembles per-image results identical to the unsharded render."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nfi import parallel


@pytest.mark.parametrize('n,ws', [(8, 2), (7, 2), (1, 2), (32, 8), (5, 3)])
def test_chunk_bounds_match_torch_chunk(n, ws):
    ref = [len(c) for c in torch.arange(n).chunk(ws)]
    got = [b - a for a, b in parallel.chunk_bounds(n, ws)]
    assert got[:len(ref)] == ref and sum(got) == n


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, n_img, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, 'tests'), root, os.path.join(root, 'nerf-from-image_amd')]
    from gpu_helpers import synthetic_inputs, run_oracle
    from nfi import parallel as par
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    torch.set_num_threads(1)
    inp, meta = synthetic_inputs(B=n_img, H=6, W=6, S=8, R=8, scene_range=1.4, seed=4)
    per_image = {k: inp[k] for k in ('planes', 'palette', 'cam', 'focal', 'u_coarse', 'g_rgb', 'g_mask')}
    mine = par.shard(per_image, rank, ws)
    a, b = par.chunk_bounds(n_img, ws)[rank]
    local = dict(inp)
    local.update(mine)
    local['u_fine'] = inp['u_fine'].view(n_img, -1, 8)[a:b].reshape(-1, 8)
    if b > a:
        out = run_oracle(local, meta)
        rows = torch.cat([out['rgb'].flatten(1), out['mask'].flatten(1), out['d_palette'].flatten(1),
                          out['d_cam'].flatten(1)], dim=1)
    else:
        rows = torch.zeros(0, 6 * 6 * 4 + 30 + 16)
    tot = par.sum_scalars([float(rows.sum()), float(b - a)], 'cpu')
    full = par.gather_rows(rows, n_img)
    if rank == 0:
        ref = run_oracle(inp, meta)
        ref_rows = torch.cat([ref['rgb'].flatten(1), ref['mask'].flatten(1), ref['d_palette'].flatten(1),
                              ref['d_cam'].flatten(1)], dim=1)
        q.put((float((full - ref_rows).abs().max()), tot[1]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('n_img,ws', [(4, 2), (3, 2)])
def test_sharded_render_equals_unsharded(n_img, ws):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, n_img, q)) for r in range(ws)]
    for p in procs:
        p.start()
    err, count = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert count == n_img
    assert err < 1e-5
