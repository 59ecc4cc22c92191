"""cProfile of the eager inversion step's host side (GPU box): which Python functions the ~14 ms of
enqueue per vgg step (B=4) go to.  Usage: python scripts/host_profile.py [loss] [steps]"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd'), os.path.join(ROOT, 'scripts')]
import torch  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import inversion, lpips, producer  # noqa: E402


def main():
    loss = sys.argv[1] if len(sys.argv) > 1 else 'vgg'
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
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
    pr = cProfile.Profile()
    pr.enable()
    inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(45)
    st.sort_stats('cumtime').print_stats(45)


if __name__ == '__main__':
    main()
