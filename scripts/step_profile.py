"""torch.profiler view of the inversion step's host side: which ops are launched how often and
what they cost on the CPU (the eager step is about as launch-bound as it is GPU-bound).
Usage (GPU box): python scripts/step_profile.py [loss] [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import inversion, lpips, producer  # noqa: E402


def main():
    loss = sys.argv[1] if len(sys.argv) > 1 else 'l1'
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device('cuda:0')
    cfg = bench.CONFIGS['p3d_fwdbwd']
    cfg = cfg[:3] + (B,) + cfg[4:]
    nfi.configure(scene_range=1.4, white_background=False, fine_sampling=True)
    batch = bench.make_inputs(cfg, dev, 1)
    torch.manual_seed(4321)
    gen = producer.InversionGenerator(scene_range=1.4).to(dev).requires_grad_(False)
    w_avg = gen.mapping_network.get_average_w(generator=torch.Generator().manual_seed(7))
    target = torch.tanh(torch.randn((B, 128, 128, 3), device=dev))
    net = lpips.LPIPS().to(dev) if loss == 'vgg' else None
    icfg = inversion.InversionConfig(steps=3, resolution=128, samples=64, loss=loss)
    inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
    torch.cuda.synchronize()
    icfg.steps = 4
    with profile(activities=[ProfilerActivity.CPU], with_stack=len(sys.argv) > 3) as prof:
        inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
        torch.cuda.synchronize()
    if len(sys.argv) > 3:            # python scripts/step_profile.py l1 4 stacks: callers of the busiest ops
        ev = prof.key_averages(group_by_stack_n=6)
        rows = sorted((e for e in ev if e.key in ('aten::mul', 'aten::copy_', 'aten::add_', 'aten::fill_', 'aten::add')),
                      key=lambda e: -e.count)[:25]
        for e in rows:
            stack = [f for f in e.stack if 'nfi' in f or 'inversion' in f or 'producer' in f][:4]
            print(f'{e.key:14s} n={e.count:4d} self={e.self_cpu_time_total:8.0f}us  ' + ' <- '.join(stack))
        return
    ev = prof.key_averages()
    print(ev.table(sort_by='self_cpu_time_total', row_limit=45))
    print(ev.table(sort_by='count', row_limit=30))


if __name__ == '__main__':
    main()
