"""Reentrancy from nn.DataParallel's per-GPU Python threads (SURVEY.md:387;
run.py:569-617 ParallelModel.forward -> render(), run in one thread per replica by
torch/nn/parallel/parallel_apply.py:114).

Two host threads, each with its own HIP stream on cuda:0, render different images forward and
backward at the same time (nfi.render through the C-ABI: no static state, the caller's stream); the
results must equal the same renders done one after the other: outputs, d palette, d cam and d focal
bit for bit (fixed-order reductions), d planes to 1e-6 relative L2 (float-atomic sums)."""

import threading

import pytest
import torch

import nfi
from gpu_helpers import rel_l2, synthetic_inputs

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def _render(inp, meta):
    planes = inp['planes'].to(DEV).requires_grad_()
    palette = inp['palette'].to(DEV).requires_grad_()
    cam = inp['cam'].to(DEV).requires_grad_()
    focal = inp['focal'].to(DEV).requires_grad_()
    f = nfi.TriplaneField(planes=planes, palette=palette, w1=inp['w1'].to(DEV), b1=inp['b1'].to(DEV),
                          w2=inp['w2'].to(DEV), b2=inp['b2'].to(DEV), alpha=float(inp['alpha']),
                          beta=float(inp['beta']))
    rgb, depth, mask, _, _, _ = nfi.render(f, meta['H'], meta['W'], cam, focal, None, None, None, meta['S'],
                                           randomize=True, u_coarse=inp['u_coarse'].to(DEV),
                                           u_fine=inp['u_fine'].to(DEV))
    ((rgb * inp['g_rgb'].to(DEV)).sum() + (mask * inp['g_mask'].to(DEV)).sum()).backward()
    return dict(rgb=rgb.detach(), depth=depth.detach(), mask=mask.detach(), d_planes=planes.grad,
                d_palette=palette.grad, d_cam=cam.grad, d_focal=focal.grad)


def test_render_from_concurrent_threads_matches_serial():
    nfi.configure(scene_range=1.4, white_background=False, fine_sampling=True, use_sdf=True,
                  attention_values=10, use_viewdir=False)
    cases = [synthetic_inputs(B=2, H=32, W=32, S=64, R=128, scene_range=1.4, seed=s) for s in (71, 72)]
    serial = []
    for inp, meta in cases:
        serial.append({k: v.cpu() for k, v in _render(inp, meta).items()})
    torch.cuda.synchronize()

    reps = 4
    results = [[None] * reps for _ in cases]
    errors = []
    barrier = threading.Barrier(len(cases))

    def worker(i):
        try:
            stream = torch.cuda.Stream(DEV)
            with torch.cuda.device(DEV), torch.cuda.stream(stream):
                barrier.wait()
                for k in range(reps):
                    out = _render(*cases[i])
                    stream.synchronize()
                    results[i][k] = {key: v.cpu() for key, v in out.items()}
        except Exception as e:  # noqa: BLE001 (re-raised in the main thread)
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(len(cases))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=200)
    assert not any(t.is_alive() for t in threads), 'a render thread hung'
    if errors:
        raise errors[0]
    for i in range(len(cases)):
        for k in range(reps):
            got = results[i][k]
            for key in ('rgb', 'depth', 'mask', 'd_palette', 'd_cam', 'd_focal'):
                assert torch.equal(got[key], serial[i][key]), (i, k, key)
            assert rel_l2(got['d_planes'], serial[i]['d_planes']) < 1e-6, (i, k)
