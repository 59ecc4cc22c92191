"""Multi-process (gloo on CPU, world_size 2 and 3) coverage of the one-process-per-GPU path
(nfi/parallel.py): the inversion batch is split with DataParallel's torch.chunk
semantics (run.py:636-640, 1757), every rank inverts its own images with nfi.inversion.invert,
and the per-image results / report rows are gathered back into batch order.

No GPU here, so the renderer inside each rank's inversion is the CPU oracle (render_fn), the
producer its PyTorch formulation; tests/test_gpu_sharded.py runs the same sharded inversion with
the HIP renderer on the GPU.  Checks: the sharded trajectory reproduces the reference's own
(tests/golden/inversion.npz, batch 2 over 2 ranks = one image per rank), and report.run over 3
images with a global batch of 2 (a tail batch of 1 leaves rank 1 empty, run.py:1879) returns the
report of the unsharded loop."""

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


def _setup_path():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, 'tests'), root, os.path.join(root, 'nerf-from-image_amd')]


def _uniforms(batches, H, S, seed):
    """Draws of a whole batch, image-major [b*H*W*S], built from per-(image, step) streams: image
    i gets the same numbers whichever batch or rank renders it.  `batches` maps a batch's first
    image to its size."""
    def fn(idx, it):
        us = [torch.rand((2, H * H * S), generator=torch.Generator().manual_seed(seed + 1000 * i + it))
              for i in range(idx, idx + batches[idx])]
        full = torch.cat(us, dim=1)
        b = batches[idx]
        return full[0].view(b, H, H, S), full[1].view(b * H * H, S)
    return fn


def _render_fn(scene_range):
    """The oracle renderer; renders without injected draws (the report's evaluation renders)
    are deterministic (randomize=False), so every process evaluates an image identically."""
    from test_producer import oracle_render_fn
    from oracle import render_oracle as orc
    inner = oracle_render_fn(scene_range)

    def fn(gen, H, W, cam, focal, center, bbox, ws, S, force_no_cam_grad=False, u_coarse=None, u_fine=None):
        if u_coarse is not None:
            return inner(gen, H, W, cam, focal, center, bbox, ws, S, force_no_cam_grad, u_coarse, u_fine)
        planes, palette = gen.planes_and_palette(ws)
        net = gen.decoder.net
        field = orc.Field(planes=planes, w1=net[0].weight, b1=net[0].bias, w2=net[2].weight, b2=net[2].bias,
                          palette=palette, alpha=gen.alpha, beta=gen.beta, scene_range=scene_range)
        return orc.render(field, H, W, cam, focal, center, bbox, S, randomize=False,
                          force_no_cam_grad=force_no_cam_grad)
    return fn


def _worker(rank, ws, port, kind, out_path):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    _setup_path()
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    from nfi import parallel as par, report
    from test_producer import inversion_setup, oracle_render_fn
    gen, d, meta, cfg = inversion_setup()
    rf = oracle_render_fn(float(meta['scene_range']))
    if kind == 'trajectory':
        res = par.invert_sharded(gen, d['target'], d['cam0'], d['focal0'], d['w_init'], cfg,
                                 uniforms=lambda it: (d['u_coarse'][it], d['u_fine'][it]),
                                 render_fn=rf)
        out = {'ws': res.ws, 'z0': res.z0, 't2': res.t2, 's': res.s, 'q': res.q,
               'losses': torch.tensor(res.losses, dtype=torch.float64)}
    else:
        cfg.steps = 2
        n = 3
        images = torch.cat([d['target'], d['target'].flip(1)])[:n]
        cams = torch.cat([d['cam0'], d['cam0'].flip(0)])[:n]
        focals = torch.cat([d['focal0'], d['focal0']])[:n]
        lines = []
        rep = report.run(gen, images, cams, focals, d['w_init'], cfg, test_bs=2,
                         report_path=os.path.join(os.path.dirname(out_path), f'ck_{rank}.pth'),
                         log=lines.append, render_fn=_render_fn(float(meta['scene_range'])), gt_cams=cams,
                         uniforms=_uniforms({0: 2, 2: 1}, int(meta['H']), int(meta['S']), 5))
        out = {f'{k}@{s}': v for s, e in rep.items() for k, v in e.items()}
        out['n_lines'] = torch.tensor(len(lines))
    torch.save(out, out_path + f'.{rank}')
    dist.barrier()
    dist.destroy_process_group()


def _spawn(ws, kind, tmp_path):
    ctx = mp.get_context('spawn')
    port = _free_port()
    out = str(tmp_path / kind)
    procs = [ctx.Process(target=_worker, args=(r, ws, port, kind, out)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return [torch.load(out + f'.{r}', weights_only=True) for r in range(ws)]


def test_sharded_inversion_reproduces_reference_trajectory(tmp_path):
    """Batch 2 over 2 ranks: each rank inverts one image.  The gathered latents / poses and the
    per-step loss sums equal one process inverting the same chunks (bit for bit, 1 thread each),
    and follow the reference's 3-step trajectory (tests/golden/inversion.npz, a batch of 2 in
    one process).  Against the golden the latent tolerance is the one of any fp32 formulation
    whose convolution rounding differs from the reference's (here: the producer's convolutions
    over 1 image instead of 2 change d ws by 3e-4 relative — the reference's own fp32 error —,
    and Adam's normalised first steps amplify that to ~1% of the displacement; the HIP loop's
    bound, tests/test_gpu_inversion.py)."""
    from test_producer import check_trajectory, inversion_setup, oracle_render_fn
    from nfi import inversion
    from nfi.inversion import InversionResult
    outs = _spawn(2, 'trajectory', tmp_path)
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k          # every rank holds the whole batch
    o = outs[0]
    res = InversionResult(ws=o['ws'], z0=o['z0'], t2=o['t2'], s=o['s'], q=o['q'], losses=o['losses'].tolist())
    gen, d, meta, cfg = inversion_setup()
    check_trajectory(res, d, loss_rtol=1e-5, w_rel=3e-2)
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        rf = oracle_render_fn(float(meta['scene_range']))
        per = [inversion.invert(gen, d['target'][i:i + 1], d['cam0'][i:i + 1], d['focal0'][i:i + 1], d['w_init'],
                                cfg, uniforms=lambda it, i=i: (d['u_coarse'][it][i:i + 1],
                                                               d['u_fine'][it][256 * i:256 * (i + 1)]),
                                render_fn=rf) for i in range(2)]
    finally:
        torch.set_num_threads(threads)
    for k in ('ws', 'z0', 't2', 's', 'q'):
        assert torch.equal(o[k], torch.cat([getattr(r, k) for r in per])), k
    ref_losses = torch.tensor([a + b for a, b in zip(per[0].losses, per[1].losses)], dtype=torch.float64)
    torch.testing.assert_close(o['losses'].double(), ref_losses, rtol=1e-12, atol=0)


def test_sharded_report_equals_unsharded(tmp_path):
    """report.run over 3 images with a global batch of 2 on 2 ranks (one image per rank; the
    tail batch of 1 runs on rank 0 alone while rank 1 joins the gathers with nothing) returns,
    on every rank, the report one process gets inverting the images one at a time with the same
    per-image draws: every row in batch order, bit for bit."""
    from nfi import report
    from test_producer import inversion_setup
    outs = _spawn(2, 'report', tmp_path)
    assert int(outs[0]['n_lines']) == 2 and int(outs[1]['n_lines']) == 0   # rank 0 logs
    gen, d, meta, cfg = inversion_setup()
    cfg.steps = 2
    n = 3
    images = torch.cat([d['target'], d['target'].flip(1)])[:n]
    cams = torch.cat([d['cam0'], d['cam0'].flip(0)])[:n]
    focals = torch.cat([d['focal0'], d['focal0']])[:n]
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        rep = report.run(gen, images, cams, focals, d['w_init'], cfg, test_bs=1,
                         report_path=str(tmp_path / 'ck_single.pth'), log=lambda s: None,
                         render_fn=_render_fn(float(meta['scene_range'])), gt_cams=cams,
                         uniforms=_uniforms({0: 1, 1: 1, 2: 1}, int(meta['H']), int(meta['S']), 5))
    finally:
        torch.set_num_threads(threads)
    ref = {f'{k}@{s}': v for s, e in rep.items() for k, v in e.items()}
    assert set(ref) == set(outs[0]) - {'n_lines'}
    for k, v in ref.items():
        assert v.shape[0] == n, k
        assert torch.equal(outs[0][k], v), k
        assert torch.equal(outs[1][k], v), k
