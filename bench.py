"""Benchmark of the nfi renderer on MI355X (driver contract: one JSON line from rank 0).

Metric (BASELINE.json): Msamples/s of the renderer fwd+bwd at 128x128, 64 coarse + 64 fine
samples per ray (sample = one radiance-field evaluation; 2,097,152 per 128^2 image).
Workload (config 'p3d_fwdbwd', default): p3d_car setting (scene_range 1.4, perspective,
camera_flipped, black background), B=8 images per GPU, the inversion step's renderer:
rays -> coarse field -> sample_pdf -> fine field -> composite, then backward to the planes,
the palette and the camera (pose).  Synthetic seeded inputs at the real sizes (planes
[8,3,32,256,256] fp32).  The tri-plane producer (synthesis network) and the LPIPS loss are
outside the timed path.

One step = one fwd+bwd render of the per-GPU batch.  Multi-GPU: one process per GPU
(torchrun), each rank renders its own images (weak scaling, no data-path collective).
"""

from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, 'nerf-from-image_amd')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # name: (scene_range, white_bg, flipped, B, H, S, pose_grad, backward)
    'p3d_fwdbwd': (1.4, False, True, 8, 128, 64, True, True),
    'p3d_fwd': (1.4, False, True, 8, 128, 64, False, False),            # BASELINE configs[1]
    'shapenet_fwdbwd': (0.55, True, False, 16, 128, 64, False, True),   # BASELINE configs[2]
    'imagenet_256': (1.4, False, True, 8, 256, 128, True, True),        # BASELINE configs[4] per GPU slice
}

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8 TB/s
TAP_BYTES = 3 * 4 * 32 * 4  # 1,536 B per sample per tap pass


def make_inputs(cfg, dev, seed):
    from nfi.synthetic import inversion_batch
    sr, wbg, flipped, B, H, S, pose, bwd = cfg
    # planes in the renderer's texel-major storage: what the producer (InversionGenerator) emits,
    # so the timed path is the inversion step's; channel-major callers pay one conversion pass each
    # way, reported separately as channel_major_conversion_ms
    return inversion_batch(B, H, H, S, 256, sr, seed, flipped=flipped, device=dev, texel_major=True)


def run_step(nfi, batch, cfg, backward: bool):
    sr, wbg, flipped, B, H, S, pose, bwd = cfg
    f = batch['field']
    f.planes.grad = None
    f.palette.grad = None
    cam = batch['cam'].detach().requires_grad_(pose and backward)
    focal = batch['focal'].detach().requires_grad_(pose and backward)
    # a forward-only step renders under no_grad, as the reference's eval renders do (run.py:2036-2051)
    with torch.enable_grad() if backward else torch.no_grad():
        rgb, depth, mask, _, _, _ = nfi.render(f, H, H, cam, focal, None, None, None, S, randomize=True)
    if backward:
        # the upstream gradients of a loss sum(rgb * g_rgb) + sum(mask * g_mask), handed in directly
        torch.autograd.backward([rgb, mask], [batch['g_rgb'], batch['g_mask']])
    return rgb


def conversion_ms(planes, ops, reps=5):
    """ms per step a caller holding channel-major [B,3,32,R,R] planes would add: the texel-major
    copy in the forward and the gradient's copy back (planes_t2c / planes_c2t)."""
    cm = planes.detach().contiguous().requires_grad_()
    g = torch.ones((cm.shape[0], 3, cm.shape[3], cm.shape[4], 32), device=cm.device)

    def once():
        cm.grad = None
        ops.planes_texel_major(cm).backward(g)
    once()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        once()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


def progress(msg: str):
    """A progress line on stderr (the JSON result alone goes to stdout)."""
    sys.stderr.write(f'[bench {time.strftime("%H:%M:%S")}] {msg}\n')
    sys.stderr.flush()


def cpu_model() -> str:
    """lscpu's 'Model name' (the /proc/cpuinfo model name when lscpu is absent)."""
    import subprocess
    try:
        out = subprocess.run(['lscpu'], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            if line.strip().startswith('Model name'):
                return line.split(':', 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 quota (cpu.max), or None when unlimited / unreadable."""
    try:
        with open('/sys/fs/cgroup/cpu.max') as fh:
            q, p = fh.read().split()[:2]
        return None if q == 'max' else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(args):
    """The CPU oracle (oracle/render_oracle.py, the reference's op graph in PyTorch) timed on this
    host's cores on a bounded sample of the same workload: ONE 128x128 image, 64+64 samples,
    fwd+bwd with plane/palette/pose gradients."""
    from oracle import render_oracle as orc
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from gpu_helpers import synthetic_inputs
    # SURVEY §8(d) CPU-baseline plan: every core this process may run on — its affinity set,
    # capped by the cgroup CPU quota where one is set (a GPU box grants each GPU's job a share of
    # the host: its affinity lists the whole machine, and threads beyond the quota only time-slice)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    share = int(math.ceil(quota)) if quota else None
    if share is None and os.environ.get('OMP_NUM_THREADS', '').isdigit():
        share = int(os.environ['OMP_NUM_THREADS'])     # the box's per-job CPU share when no quota is visible
    cores = max(1, min(affinity, share) if share else affinity)
    torch.set_num_threads(cores)
    progress(f'cpu baseline: {cores} threads (affinity {affinity}, cgroup quota {quota})')
    H = args.cpu_res
    inp, meta = synthetic_inputs(B=1, H=H, W=H, S=64, R=256, scene_range=1.4, seed=0)
    field = orc.Field(planes=inp['planes'].clone().requires_grad_(), w1=inp['w1'], b1=inp['b1'],
                      w2=inp['w2'], b2=inp['b2'], palette=inp['palette'].clone().requires_grad_(),
                      alpha=inp['alpha'], beta=inp['beta'], scene_range=1.4)

    def once():
        cam = inp['cam'].clone().requires_grad_()
        focal = inp['focal'].clone().requires_grad_()
        rgb, depth, mask = orc.render(field, H, H, cam, focal, None, None, 64, randomize=True)
        ((rgb * inp['g_rgb']).sum() + (mask * inp['g_mask']).sum()).backward()

    once()  # warm-up
    times = []
    for k in range(args.cpu_reps):
        t0 = time.perf_counter()
        once()
        times.append(time.perf_counter() - t0)
        progress(f'cpu baseline rep {k}: {times[-1]:.2f} s')
    t = sorted(times)[len(times) // 2]
    samples = H * H * 128
    model = cpu_model()
    out = {'value': samples / t / 1e6, 'unit': 'Msamples/s', 'cores': cores, 'kind': 'port',
           'sample': f'1 image {H}x{H}, 64+64 samples/ray, fwd+bwd (planes, palette, pose grads), '
                     f'median of {args.cpu_reps} after 1 warm-up; torch.set_num_threads({cores}) = '
                     f'min(len(sched_getaffinity) {affinity}, the CPU share granted: cgroup quota {quota} / '
                     f'OMP_NUM_THREADS {os.environ.get("OMP_NUM_THREADS")}); {model}',
           'affinity_cpus': affinity,
           'cpu_model': model, 'cgroup_cpu_quota': cgroup_cpu_quota(),
           'reps_seconds': [round(x, 3) for x in times],
           'seconds_per_image_step': t}
    if not args.no_inversion:
        inv = cpu_inversion_step(inp, H, args.inv_loss.split(','))
        first = args.inv_loss.split(',')[0]
        out['inversion'] = inv[first]
        for k, v in inv.items():
            if k != first:
                out[f'inversion_{k}'] = v
    return out


def cpu_inversion_step(inp, H, loss_kinds):
    """One step of the inversion loop on the CPU, the reference's way: the producer's reference op
    sequence in PyTorch (oracle/producer_oracle.py) + the oracle renderer, the loss, Adam; 1 image at
    HxH, 64+64 samples; s/image for 30 steps = 30 x the step (timed after one warm-up step)."""
    from nfi import inversion, lpips, producer
    from oracle import producer_oracle as po
    from oracle import render_oracle as orc
    torch.manual_seed(4321)
    gen = producer.InversionGenerator(scene_range=1.4)
    with torch.no_grad():
        gen.decoder.net[2].bias[0] -= 0.97
    gen.requires_grad_(False)
    gen = po.ReferenceProducer(gen)
    w_avg = gen.mapping_network.get_average_w(n_samples=1000, generator=torch.Generator().manual_seed(7))
    target = torch.tanh(torch.randn((1, H, H, 3), generator=torch.Generator().manual_seed(99)))

    def render_fn(g, Hh, Ww, cam, focal, center, bbox, ws, S, force_no_cam_grad=False, **kw):
        planes, palette = g.planes_and_palette(ws)
        net = g.decoder.net
        field = orc.Field(planes=planes, w1=net[0].weight, b1=net[0].bias, w2=net[2].weight,
                          b2=net[2].bias, palette=palette, alpha=g.alpha, beta=g.beta, scene_range=1.4)
        return orc.render(field, Hh, Ww, cam, focal, center, bbox, S, randomize=True,
                          force_no_cam_grad=force_no_cam_grad)

    res = {}
    for loss in loss_kinds:
        progress(f'cpu inversion step ({loss})')
        cfg = inversion.InversionConfig(steps=1, resolution=H, samples=64, loss=loss, camera_flipped=True)
        net = po.ReferenceLPIPS(lpips.LPIPS()) if loss in inversion.VGG_LOSSES else None
        inversion.invert(gen, target, inp['cam'], inp['focal'], w_avg, cfg, render_fn=render_fn, lpips_net=net)
        t0 = time.perf_counter()
        inversion.invert(gen, target, inp['cam'], inp['focal'], w_avg, cfg, render_fn=render_fn, lpips_net=net)
        step = time.perf_counter() - t0
        res[loss] = {'s_per_image': round(30 * step, 3), 'step_seconds': round(step, 3),
                     'sample': f'1 image {H}x{H}, 64+64 samples, producer (oracle: reference op sequence) + oracle render '
                               f'fwd+bwd, loss {loss}, Adam; one timed step after one warm-up, x30'}
    return res


def max_over_ranks(x: float, dev) -> float:
    """MAX of a host float over the ranks (on the device for RCCL, on the host for gloo)."""
    t = torch.tensor([x], device=dev if dist.get_backend() == 'nccl' else 'cpu', dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def inversion_leg(args, dev, cfg, world, loss):
    """BASELINE.json's second number: seconds per image of the 30-step inversion (run.py:1960-2310,
    pose optimised), BASELINE configs[3]: a global batch of --inv-batch images per GPU (4: 32 over 8
    GPUs) split over the ranks by nfi.parallel.invert_sharded (DataParallel's torch.chunk,
    run.py:636-640, 1757; every rank holds the whole batch's targets and cameras, inverts its
    chunk, and the per-image results are all_gathered — over RCCL under torchrun).  Per step the
    producer (synthesis network + AttentionMapper, fp32), the HIP render fwd+bwd, the loss ('vgg' =
    the reference default --inv_loss: LPIPS-VGG over the image + 15 augmented copies, random
    weights since none ship offline; or 'l1'), the backward to the latent and pose, Adam.
    Random-init generator (no checkpoint offline), z_avg from the mapping network, seeded cameras
    (nfi.synthetic.cameras), a synthetic target image.  Timed like the renderer leg (barrier +
    synchronize around exactly --inv-steps steps, max over ranks); the final all_gather of the
    results is inside the timed region."""
    from nfi import conv as _conv, inversion, lpips, ops, parallel, producer, synthetic
    sr, wbg, flipped, _, H, S, pose, bwd = cfg
    progress(f'inversion leg ({loss})')
    B = args.inv_batch * world      # the global step batch
    torch.manual_seed(4321)
    gen = producer.InversionGenerator(scene_range=sr).to(dev)
    with torch.no_grad():
        gen.decoder.net[2].bias[0] -= 0.97        # the synthetic field's SDF shift (nfi/synthetic.py)
    gen.requires_grad_(False)
    w_avg = gen.mapping_network.get_average_w(generator=torch.Generator().manual_seed(7))
    g = torch.Generator(device=dev).manual_seed(99)
    target = torch.tanh(torch.randn((B, H, H, 3), generator=g, device=dev))
    cam, focal = synthetic.cameras(B, sr, 4321, flipped=flipped, device=dev)
    icfg = inversion.InversionConfig(steps=2, resolution=H, samples=S, loss=loss,
                                     camera_flipped=flipped, white_background=wbg,
                                     graph=args.inv_graph)
    net = lpips.LPIPS().to(dev) if loss in inversion.VGG_LOSSES else None
    # warm-up: library plans (MIOpen / hipBLASLt), frozen-weight caches, and the step's HIP graph
    # (captured after inversion.EAGER_STEPS eager steps; the timed batch reuses it, as every later
    # batch of a run does)
    icfg.steps = inversion.EAGER_STEPS + 1 if icfg.graph else 2
    parallel.invert_sharded(gen, target, cam, focal, w_avg, icfg, lpips_net=net)
    # the renderer's share: HIP events over one further eager step (first-launch costs excluded)
    ops.KERNEL_TIMERS = {}
    icfg.steps = 1
    parallel.invert_sharded(gen, target, cam, focal, w_avg, icfg, lpips_net=net)
    torch.cuda.synchronize()
    timers, ops.KERNEL_TIMERS = ops.KERNEL_TIMERS, None
    render_ms = sum(a.elapsed_time(b) for v in timers.values() for a, b in v)
    icfg.steps = args.inv_steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = parallel.invert_sharded(gen, target, cam, focal, w_avg, icfg, lpips_net=net)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev)
    step_ms = elapsed / icfg.steps * 1e3
    # s/image of a 30-step inversion (run.py:1829-1830: checkpoint_steps [0, 30] by default): all ranks
    # together finish the B-image batch in `elapsed` for icfg.steps steps
    return {'s_per_image': round(elapsed * 30 / icfg.steps / B, 5), 'steps': icfg.steps,
            'images': B, 'images_per_gpu': args.inv_batch, 'seconds': round(elapsed, 4),
            'ms_per_step': round(step_ms, 3),
            'render_ms_per_step': round(render_ms, 3),
            'rest_ms_per_step': round(step_ms - render_ms, 3),
            'sharding': f'nfi.parallel.invert_sharded: {B} images over {world} rank(s), torch.chunk, '
                        f'results all_gathered ({dist.get_backend() if world > 1 else "single process"})',
            'loss': loss + (' (LPIPS-VGG, random weights, 16 copies; parity unpinned: no lpips weights or '
                                   'package offline)' if net is not None else ''),
            'loss_first_last': [round(res.losses[0], 5), round(res.losses[-1], 5)],
            'producer': 'StyleGAN2 synthesis 256^2x96 + AttentionMapper, fp32: 3x3 convs Winograd F(4,3) '
                        + ('(nfi HIP transforms + nfi split-f16 batched GEMM, fp32-accurate), up-sampling convs as one '
                           '9-tap GEMM (split-f16 for maps >= 32^2, else hipBLASLt) + HIP FIR, '
                           if _conv.SPLIT16 else '(nfi HIP transforms + hipBLASLt batched GEMM), up-sampling convs as '
                                                 'one 9-tap GEMM + HIP FIR, ')
                        + 'epilogues/FIR/skip/modulation-backward nfi HIP',
            'renderer': 'nfi HIP fwd+bwd',
            'step_replay': ('HIP graph of the whole step (captured in the warm-up batch, reused)'
                            if icfg.graph else 'eager launches')}


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` started without torchrun (WORLD_SIZE unset): start N rank processes of
    this script, one per GPU, torchrun-style (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), before
    anything here touches the GPU, wait for them and return the worst exit code.  Refuses when
    the node has fewer devices than ranks (RCCL needs one GPU per rank): it never reports a run
    of fewer GPUs under n_gpus N."""
    import subprocess
    backend = os.environ.get('NFI_BENCH_DIST', 'nccl')
    ndev = torch.cuda.device_count()     # counting devices does not initialise the GPU
    if backend == 'nccl' and ndev < n:
        sys.stderr.write(f'bench.py: --gpus {n} needs {n} visible GPUs, found {ndev}\n')
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        sys.stderr.write(f'bench.py: rank exit codes {rcs}\n')
        return bad[0] if bad[0] > 0 else 1
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--config', default='p3d_fwdbwd', choices=sorted(CONFIGS))
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-reps', type=int, default=3)
    ap.add_argument('--cpu-res', type=int, default=128)
    ap.add_argument('--no-inversion', action='store_true')
    ap.add_argument('--no-configs', action='store_true', help='time only --config (no other configs[] sub-objects)')
    ap.add_argument('--inv-steps', type=int, default=30)
    ap.add_argument('--inv-batch', type=int, default=4, help='images per GPU in the inversion leg')
    ap.add_argument('--inv-graph', action='store_true',
                    help='inversion leg with the step replayed as a HIP graph (measured slower; off)')
    ap.add_argument('--inv-loss', default='vgg,l1',
                    help="comma list; the first is reported as inversion_s_per_image")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error('--gpus must be >= 1')
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        ap.error(f'--gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU)')
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # NFI_BENCH_DIST=gloo rehearses the N-rank path on a box with fewer GPUs than ranks (ranks
    # share devices round-robin); the driver's multi-GPU runs use RCCL ('nccl'), one GPU per rank.
    backend = os.environ.get('NFI_BENCH_DIST', 'nccl')
    if backend != 'nccl':
        local = local % max(1, torch.cuda.device_count())
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group(backend, **({'device_id': dev} if backend == 'nccl' else {}))

    import nfi
    from nfi import ops
    out = measure(args.config, args, nfi, ops, dev, world, rank, headline=True)
    sr, wbg, flipped, B, H, S, pose, bwd = CONFIGS[args.config]
    if args.config == 'p3d_fwdbwd' and not args.no_configs:
        # the other single-GPU configurations of BASELINE.json, each its own timed loop (parity-test
        # cases too; the headline stays p3d_fwdbwd)
        out['configs'] = {name: measure(name, args, nfi, ops, dev, world, rank, headline=False)
                          for name in ('p3d_fwd', 'shapenet_fwdbwd', 'imagenet_256')}
    if bwd and not args.no_inversion:
        for k, loss in enumerate(args.inv_loss.split(',')):
            leg = inversion_leg(args, dev, CONFIGS[args.config], world, loss)
            out['inversion' if k == 0 else f'inversion_{loss}'] = leg
            if k == 0:
                out['inversion_s_per_image'] = leg['s_per_image']
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(args)
        out['cpu_baseline'] = cb
        out['speedup_vs_cpu'] = round(out['value'] / cb['value'], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


# fp32 FLOPs per sample: forward 6,450 (5,504 of them the decoder on MFMA); field
# backward 5,700 (5,504 MFMA); tile pass 768 per tap pass (d planes; + 768 for the grid gradients)
FLOPS = {'render_fwd': (6450, 5504), 'bwd_bins': (0, 0), 'bwd_field': (5700, 5504)}
KERNEL_OF = {'render_fwd': 'render_fwd_kernel', 'bwd_field': 'field_bwd_kernel',
             'bwd_tiles': 'tile_kernel', 'bwd_bins': 'scan_blocks_kernel'}
# gather ceiling of the FORWARD's own tap stream, measured: the product gather alone over the
# forward's merged samples at its occupancy (scripts/gather_probe.py, profiles/r03_gather_probe.json:
# 0.865 ms for 25.8 GB of taps; L1 hits on top of MI355X_MICROARCH.md's 16.8-18.8 TB/s from L2).
# Reported only for render_fwd: no other kernel's access pattern was measured against it.
GATHER_CEILING_GBS = 29790.0


def compulsory_bytes(name, pose, H, S):
    """SURVEY §8(d) compulsory HBM bytes per sample of each launch: the planes read once per image and
    tap pass (25.17 MB = 12 B per sample at 128^2 x 128), d planes written once; nothing else a launch
    handles is compulsory (the per-sample intermediates are this design's, per-ray I/O < 0.5 B)."""
    plane = 3 * 32 * 256 * 256 * 4 / (H * H * 2 * S)
    return {'render_fwd': plane, 'bwd_bins': 0.0, 'bwd_field': 0.0,
            # d planes written once + (pose gradients) the planes read once for the grid gradients
            'bwd_tiles': plane * (2 if pose else 1)}[name]


def hbm_model(name, pose, bwd, H, S):
    """This DESIGN's streamed HBM bytes per sample of each launch: the compulsory
    bytes plus the per-sample state the design moves between launches."""
    plane = compulsory_bytes('render_fwd', pose, H, S)
    return {
        # planes + saved state written (t, sigma 8 B, rgb 12, decoder outputs 44, inputs 128, perm 2)
        'render_fwd': plane + (194 if bwd else 0),
        'bwd_bins': 12.0,
        # saved state read (194) + feature-gradient row written (128) + 3 entry records (48) + 8
        'bwd_field': 194 + 128 + 48 + 8,
        # compulsory (d planes, planes for the grid gradients) + the sample's 128-B gradient row read
        # once per plane (3x: the three planes' tiles of a sample are different tiles) + its three 16-B
        # records + (pose) the 24-B grid-gradient row written
        'bwd_tiles': compulsory_bytes('bwd_tiles', pose, H, S) + 3 * 128 + 48 + (24 if pose else 0),
    }[name]


def measure(name, args, nfi, ops, dev, world, rank, headline):
    """One configuration's timed loop: --warmup untimed steps, then exactly --steps steps bracketed
    by barrier + synchronize, max over ranks; per-stage HIP-event times on the launch streams."""
    cfg = CONFIGS[name]
    sr, wbg, flipped, B, H, S, pose, bwd = cfg
    progress(f'config {name}')
    nfi.configure(scene_range=sr, white_background=wbg, fine_sampling=True)
    batch = make_inputs(cfg, dev, seed=1234 + rank)
    steps = args.steps if headline else max(3, min(args.steps, 10))
    for _ in range(args.warmup if headline else 2):
        run_step(nfi, batch, cfg, bwd)
    torch.cuda.synchronize()
    ops.KERNEL_TIMERS = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run_step(nfi, batch, cfg, bwd)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timers, ops.KERNEL_TIMERS = ops.KERNEL_TIMERS, None
    # ms per step of each stage: the sum of its launches
    kern = {k: sum(a.elapsed_time(b) for a, b in v) / steps for k, v in timers.items()}
    launches = {k: len(v) / steps for k, v in timers.items()}
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev)
    samples_per_step = B * H * H * 2 * S
    value = world * samples_per_step * steps / elapsed / 1e6
    ms_per_step = elapsed / steps * 1e3
    conv_ms = conversion_ms(batch['field'].planes, ops) if headline else None
    del batch
    torch.cuda.empty_cache()

    tap = {'render_fwd': TAP_BYTES, 'bwd_bins': 0, 'bwd_field': 0,
           'bwd_tiles': TAP_BYTES * (2 if pose else 1)}
    flops = dict(FLOPS, bwd_tiles=(768 * (2 if pose else 1), 0))
    stages = {}
    for k, v in kern.items():
        if k not in tap:
            continue
        sec = v * 1e-3 / launches[k]
        per_launch = samples_per_step / launches[k]
        stages[k] = {'ms': round(v, 4), 'launches_per_step': launches[k],
                     'compulsory_bytes_per_sample': round(compulsory_bytes(k, pose, H, S), 2),
                     'compulsory_GBps': round(per_launch * compulsory_bytes(k, pose, H, S) / sec / 1e9, 1),
                     'design_stream_bytes_per_sample': round(hbm_model(k, pose, bwd, H, S), 1),
                     'design_stream_GBps': round(per_launch * hbm_model(k, pose, bwd, H, S) / sec / 1e9, 1),
                     'tap_rate_GBps': round(per_launch * tap[k] / sec / 1e9, 1),
                     'fp32_TFLOPs': round(per_launch * flops[k][0] / sec / 1e12, 2),
                     'mfma_TFLOPs': round(per_launch * flops[k][1] / sec / 1e12, 2)}
    res = {'metric': (f'Msamples/sec fwd+bwd ({H}^2, {S}+{S} samples/ray)' if bwd
                      else f'Msamples/sec fwd ({H}^2, {S}+{S} samples/ray)'),
           'value': round(value, 3), 'unit': 'Msamples/s', 'n_gpus': world, 'steps': steps,
           'warmup': args.warmup if headline else 2, 'ms_per_step': round(ms_per_step, 4),
           'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
           'dtype': 'f32 (decoder: 3-term split-f16 MFMA)',
           'data': 'synthetic',
           'config': {'workload': name, 'global_batch': B * world, 'resolution': H,
                      'samples_per_ray': f'{S}+{S}', 'plane_res': 256, 'pose_grad': pose,
                      'backward': bwd, 'white_background': wbg, 'scene_range': sr,
                      'parallelism': f'dp{world} (one process per GPU, no collective)',
                      'planes_layout': 'texel-major [B,3,R,R,32] storage (the producer\'s native output)'},
           'renderer_s_per_image_30step': round(30 * ms_per_step / 1e3 / B, 5),
           'stages': stages}
    if not headline:
        for key in ('metric', 'unit', 'n_gpus', 'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'data'):
            res.pop(key)
        return res
    res['channel_major_conversion_ms'] = conv_ms

    # roofline of the dominant launch (the longest HIP-event-timed stage)
    dom = max(stages, key=lambda k: stages[k]['ms'] / stages[k]['launches_per_step'])
    st = stages[dom]
    sec = st['ms'] * 1e-3 / st['launches_per_step']
    per_launch = samples_per_step / st['launches_per_step']
    traffic, traffic_src, counters = None, 'none', None
    try:
        from nfi.build import source_digest
        with open(os.path.join(ROOT, 'profiles', 'latest_counters.json')) as fh:
            cj = json.load(fh)
        ctr = cj['kernels'].get(KERNEL_OF[dom])
        if cj.get('source_digest') != source_digest():
            traffic_src = f"stale ({cj.get('tag')}: counters of other kernel sources; not used)"
        elif ctr is not None and name == cj.get('config', 'p3d_fwdbwd') and B == cj.get('batch', 8):
            traffic = round(ctr['hbm_bytes_corrected'] / 1e9, 3)
            traffic_src = (f"profiles/latest_counters.json ({cj.get('tag')}, source digest {cj['source_digest']}): "
                           f"rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate passes")
            # the same profile's SQ / TCC passes for this kernel (scripts/summarize_round.py):
            # matrix-pipe busy share and EXECUTED MFMA rate (incl. the backward's layer-1
            # recompute and the padded output block), VALU issue share, L2 hit rate
            counters = {k: round(ctr[k], 4) for k in ('mfma_busy', 'mfma_TFLOPs', 'mfma_flop_frac',
                                                      'valu_issue_share', 'waves_per_simd',
                                                      'issue_stall_share', 'l2_hit', 'avg_us')
                        if ctr.get(k) is not None}
    except (OSError, ValueError, KeyError):
        pass
    # the decoder's matrix-core utilisation (north star: "MFMA utilisation for the MLP against gfx950
    # peak"): per decoder launch, live HIP-event fp32-work rate of the reference MLP's FLOPs, and the
    # same profile's counters (executed f16 MFMA rate; the split-f16 decoder does three f16 products
    # per fp32 product)
    decoder = {}
    for stg in ('render_fwd', 'bwd_field'):
        if stg not in stages:
            continue
        # fp32_work: the reference MLP's 5,504 FLOP per sample / launch time, against the
        # fp32 peak; f16_pipe: the same work as the three f16 products per fp32 product the split needs,
        # against the f16 matrix peak (counters_*: EXECUTED f16 MFMAs incl. recompute and padding)
        ent = {'fp32_work_TFLOPs': stages[stg]['mfma_TFLOPs'],
               'fp32_work_frac': round(stages[stg]['mfma_TFLOPs'] / 157.3, 4), 'fp32_peak_TFLOPs': 157.3,
               'f16_pipe_frac': round(3 * stages[stg]['mfma_TFLOPs'] / 2500.0, 4), 'f16_peak_TFLOPs': 2500.0}
        try:
            if cj.get('source_digest') == source_digest():
                c2 = cj['kernels'].get(KERNEL_OF[stg], {})
                for key in ('mfma_f16_exec_TFLOPs', 'mfma_f16_exec_frac', 'mfma_busy', 'valu_issue_share'):
                    if c2.get(key) is not None:
                        ent['counters_' + key] = round(c2[key], 4)
                ent['counters_f16_peak_TFLOPs'] = 2500.0
        except (NameError, KeyError, AttributeError, TypeError):
            pass
        decoder[KERNEL_OF[stg]] = ent
    res['decoder_mfma'] = dict(decoder, dtype='fp32 operands as hi/lo fp16 pairs on v_mfma_f32_16x16x32_f16 '
                                     '(three products per fp32 product; fp32-accurate, DESIGN.md §3)')
    # roofline of the dominant launch (DESIGN.md §5 gives each formula):
    #   achieved = SURVEY §8(d) compulsory bytes per sample x samples per launch / HIP-event launch time
    #   tap_rate = §8(d) tap bytes per sample (1,536 per tap pass) x samples / time: an effective rate
    #              that exceeds the HBM peak where L2 / the Infinity Cache serve the taps
    #   traffic  = rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE per launch (profiles/latest_counters.json; the
    #              counters include Infinity-Cache hits), and its ratio to the compulsory bytes
    #   design_stream = this design's streamed bytes (hbm_model) / time
    comp_b = compulsory_bytes(dom, pose, H, S)
    comp_bytes = per_launch * comp_b
    achieved = comp_bytes / sec / 1e9
    model_bytes = per_launch * hbm_model(dom, pose, bwd, H, S)
    tap_b = tap[dom]
    roof = {
        'bound': 'hbm', 'kernel': KERNEL_OF[dom], 'stage': dom,
        'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
        'frac': round(achieved / HBM_PEAK_GBS, 4),
        'frac_basis': (f'SURVEY §8(d) compulsory bytes {comp_b:.1f} B/sample (planes read once per image and tap '
                       f'pass, d planes written once) x {per_launch:.0f} samples / HIP-event launch time'),
        'traffic': traffic, 'traffic_unit': 'GB per launch', 'traffic_source': traffic_src,
        'traffic_over_compulsory': (round(traffic * 1e9 / comp_bytes, 1) if traffic is not None and comp_bytes > 0
                                    else None),
        'traffic_GBps': round(traffic / sec, 1) if traffic is not None else None,
        'traffic_frac': round(traffic / sec / HBM_PEAK_GBS, 4) if traffic is not None else None,
        'launch_ms': round(sec * 1e3, 4),
        'compulsory_bytes_per_sample': round(comp_b, 2),
        'tap_bytes_per_sample': tap_b,
        'tap_rate_GBps': st['tap_rate_GBps'],
        'tap_rate_over_hbm_peak': round(st['tap_rate_GBps'] / HBM_PEAK_GBS, 4),
        'design_stream_bytes_per_sample': round(hbm_model(dom, pose, bwd, H, S), 1),
        'design_stream_GBps': round(model_bytes / sec / 1e9, 1),
        'design_stream_frac': round(model_bytes / sec / 1e9 / HBM_PEAK_GBS, 4),
        'fp32_TFLOPs': st['fp32_TFLOPs'], 'fp32_peak_TFLOPs': 157.3,
        'fp32_frac': round(st['fp32_TFLOPs'] / 157.3, 4),
        'fp32_basis': 'SURVEY §8(d) algorithmic fp32 FLOPs per sample / HIP-event launch time',
        'counters': counters,
    }
    if dom == 'render_fwd':
        roof['gather_ceiling_GBps'] = GATHER_CEILING_GBS
        roof['gather_ceiling_frac'] = round(st['tap_rate_GBps'] / GATHER_CEILING_GBS, 4)
    res['roofline'] = roof
    return res


if __name__ == '__main__':
    main()
