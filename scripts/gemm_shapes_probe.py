"""Device time of the inversion step's generic PyTorch GEMMs (mm / bmm / addmm / baddbmm / linear)
by input shapes (GPU box), to find the small products that run on a few workgroups for long.
Usage: python scripts/gemm_shapes_probe.py [loss] [steps] [all]  ('all': every op, not only GEMMs)"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd'), os.path.join(ROOT, 'scripts')]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import inversion, lpips, producer  # noqa: E402

GEMMS = ('aten::mm', 'aten::bmm', 'aten::addmm', 'aten::baddbmm', 'aten::baddbmm_', 'aten::linear', 'aten::matmul')


def main():
    loss = sys.argv[1] if len(sys.argv) > 1 else 'l1'
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    every = len(sys.argv) > 3 and sys.argv[3] == 'all'
    dev = torch.device('cuda:0')
    B = 4
    cfg = bench.CONFIGS['p3d_fwdbwd']
    cfg = cfg[:3] + (B,) + cfg[4:]
    nfi.configure(scene_range=1.4, white_background=False, fine_sampling=True)
    batch = bench.make_inputs(cfg, dev, 1)
    torch.manual_seed(4321)
    gen = producer.InversionGenerator(scene_range=1.4).to(dev).requires_grad_(False)
    w_avg = gen.mapping_network.get_average_w(generator=torch.Generator().manual_seed(7))
    target = torch.tanh(torch.randn((B, 128, 128, 3), device=dev))
    net = lpips.LPIPS().to(dev) if loss == 'vgg' else None
    icfg = inversion.InversionConfig(steps=inversion.EAGER_STEPS + 1, resolution=128, samples=64, loss=loss)
    inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
    torch.cuda.synchronize()
    icfg.steps = steps
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key in GEMMS or (every and e.key.startswith('aten::') and e.device_time_total > 0):
            k = (e.key, str(e.input_shapes))
            agg[k][0] += e.count
            agg[k][1] += e.device_time_total
    for (name, shapes), (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60 if every else 30]:
        print(f'{t / steps / 1e3:8.3f} ms/step  {cnt / steps:5.1f}/step  {name:14s} {shapes}')


if __name__ == '__main__':
    main()
