"""Renderer fwd+bwd steps of bench.py's p3d_fwdbwd workload for LDS counter passes (GPU box):
POSE=0 renders without the pose gradient (the tile pass then skips its per-entry grid gradients,
entry_grid_grad), so the two runs' SQ_LDS_BANK_CONFLICT of tile_kernel separate that stage's
conflicts from the row staging's.
Usage: POSE=0|1 python scripts/lds_probe.py [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd')]
import torch  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    pose = os.environ.get('POSE', '1') == '1'
    cfg = bench.CONFIGS['p3d_fwdbwd']
    cfg = cfg[:6] + (pose,) + cfg[7:]
    dev = torch.device('cuda:0')
    nfi.configure(scene_range=cfg[0], white_background=cfg[1], fine_sampling=True)
    batch = bench.make_inputs(cfg, dev, 1)
    for _ in range(steps):
        bench.run_step(nfi, batch, cfg, True)
    torch.cuda.synchronize()
    print(f'lds_probe pose={pose} steps={steps} ok')


if __name__ == '__main__':
    main()
