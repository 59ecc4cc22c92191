"""Probe of the inversion step on one GPU: wall time per step vs GPU time, CPU enqueue time,
batch scaling, LPIPS memory format.  Usage (GPU box): python scripts/inversion_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import inversion, lpips, producer  # noqa: E402


def run(B, loss, steps=10, cl=False, graph=False, overlap=True):
    dev = torch.device('cuda:0')
    cfg = bench.CONFIGS['p3d_fwdbwd']
    cfg = cfg[:3] + (B,) + cfg[4:]
    nfi.configure(scene_range=1.4, white_background=False, fine_sampling=True)
    batch = bench.make_inputs(cfg, dev, 1)
    torch.manual_seed(4321)
    gen = producer.InversionGenerator(scene_range=1.4).to(dev).requires_grad_(False)
    if os.environ.get('NFI_PLANES_LAYOUT'):    # A/B: 'nchw' = channel-major planes (converted by render)
        for m in gen.modules():
            if isinstance(m, producer.ToPlanes):
                m.out_layout = os.environ['NFI_PLANES_LAYOUT']
    w_avg = gen.mapping_network.get_average_w(generator=torch.Generator().manual_seed(7))
    target = torch.tanh(torch.randn((B, 128, 128, 3), device=dev))
    net = lpips.LPIPS().to(dev) if loss == 'vgg' else None
    if net is not None and cl:
        net = net.to(memory_format=torch.channels_last)
    icfg = inversion.InversionConfig(steps=inversion.EAGER_STEPS + 1, resolution=128, samples=64, loss=loss,
                                     graph=graph, overlap_target=overlap)
    inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
    torch.cuda.synchronize()
    icfg.steps = steps
    enq = []
    t0 = time.perf_counter()
    inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net,
                     on_step=lambda it, l: enq.append(time.perf_counter()))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    cpu = (enq[-1] - enq[0]) / (steps - 1)
    print(f'B={B:3d} loss={loss:4s} cl={cl} graph={graph} overlap={overlap}: {wall * 1e3:7.2f} ms/step  {wall * 30 / B:.4f} s/img  '
          f'(enqueue {cpu * 1e3:.2f} ms/step between on_step calls)', flush=True)


if os.environ.get('NFI_BLAS'):         # A/B of the BLAS backend behind torch.bmm / mm ('cublas' = rocBLAS)
    torch.backends.cuda.preferred_blas_library(os.environ['NFI_BLAS'])

if __name__ == '__main__':
    if len(sys.argv) > 1:          # python scripts/inversion_probe.py B loss steps
        run(int(sys.argv[1]), sys.argv[2], steps=int(sys.argv[3]), graph=os.environ.get('NFI_GRAPH') == '1')
        sys.exit(0)
    for loss in ('l1', 'vgg'):
        for graph in (False, True):
            for overlap in ((True, False) if loss == 'vgg' else (True,)):
                run(4, loss, steps=30, graph=graph, overlap=overlap)
