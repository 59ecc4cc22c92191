"""The sharded inversion on the GPU (nfi/parallel.py): two rank processes share
cuda:0 under a gloo process group (the box has one GPU; the driver's multi-GPU runs use RCCL, one
GPU per rank), each inverting its torch.chunk of the batch with the HIP renderer and producer,
and the results gathered in batch order.

Checks against (1) the reference's 3-step trajectory (tests/golden/inversion.npz, batch 2 = one
image per rank) at the HIP loop's tolerance (tests/test_gpu_inversion.py) and (2) this process
inverting the same chunks one after the other on the same GPU (the unsharded computation of each
image; the HIP d-planes sums are deterministic, the producer's GEMMs run on the same shapes)."""

import os
import socket
import subprocess
import sys

import pytest
import torch

import nfi
from nfi import inversion
from nfi.inversion import InversionResult
from test_producer import check_trajectory, inversion_setup

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys
root = sys.argv[1]
sys.path[:0] = [os.path.join(root, 'tests'), root, os.path.join(root, 'nerf-from-image_amd')]
import torch
import torch.distributed as dist
import nfi
from nfi import parallel
from test_producer import inversion_setup
dist.init_process_group('gloo')
dev = torch.device('cuda:0')
gen, d, meta, cfg = inversion_setup(dev)
nfi.configure(scene_range=float(meta['scene_range']), white_background=False, fine_sampling=True,
              use_sdf=True, attention_values=10, use_viewdir=False)
res = parallel.invert_sharded(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg,
                              uniforms=lambda it: (d['u_coarse'][it], d['u_fine'][it]))
torch.save({'ws': res.ws.cpu(), 'z0': res.z0.cpu(), 't2': res.t2.cpu(), 's': res.s.cpu(), 'q': res.q.cpu(),
            'losses': torch.tensor(res.losses, dtype=torch.float64)}, sys.argv[2] + '.' + os.environ['RANK'])
dist.barrier()
dist.destroy_process_group()
'''


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_hip_inversion(tmp_path):
    ws = 2
    script = tmp_path / 'worker.py'
    script.write_text(WORKER)
    out = str(tmp_path / 'res')
    port = _free_port()
    procs = []
    for r in range(ws):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(ws), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script), ROOT, out], env=env))
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * ws, rcs
    outs = [torch.load(f'{out}.{r}', weights_only=True) for r in range(ws)]
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k            # every rank holds the whole batch
    o = outs[0]
    res = InversionResult(ws=o['ws'], z0=o['z0'], t2=o['t2'], s=o['s'], q=o['q'], losses=o['losses'].tolist())
    dev = torch.device('cuda:0')
    gen, d, meta, cfg = inversion_setup(dev)
    d_cpu = {k: v.cpu() for k, v in d.items()}
    rel = check_trajectory(res, d_cpu, loss_rtol=1e-4, w_rel=1.5e-2)
    print(f'sharded HIP inversion: latent distance / reference displacement {rel:.2e}')
    # the same chunks inverted one after the other in this process
    nfi.configure(scene_range=float(meta['scene_range']), white_background=False, fine_sampling=True,
                  use_sdf=True, attention_values=10, use_viewdir=False)
    per = [inversion.invert(gen, d['target'][i:i + 1], d['cam0'][i:i + 1], d['focal0'][i:i + 1], d['w_init'], cfg,
                            uniforms=lambda it, i=i: (d['u_coarse'][it][i:i + 1], d['u_fine'][it][256 * i:256 * (i + 1)]))
           for i in range(2)]
    moved = float((d_cpu['ws'] - d_cpu['w_init']).norm())
    seq_ws = torch.cat([r.ws.cpu() for r in per])
    assert float((seq_ws - o['ws']).norm()) < 1e-3 * moved
    for k in ('z0', 't2', 's', 'q'):
        torch.testing.assert_close(torch.cat([getattr(r, k).cpu() for r in per]), o[k], rtol=1e-5, atol=1e-6)
    seq_losses = torch.tensor([a + b for a, b in zip(per[0].losses, per[1].losses)], dtype=torch.float64)
    torch.testing.assert_close(o['losses'], seq_losses, rtol=1e-6, atol=0)
