"""Cell-run statistics of the tile pass's entry lists (GPU box): one p3d_fwdbwd step of bench.py's
workload, the backward's workspace kept (nfi.ops.DEBUG_BACKWARD), the bin list read back and split
the way tile_chunk splits it (chunks of CHUNK entries per tile, four wave ranges per chunk, per =
ceil(n/4) rounded up to 8).  Prints the share of entries whose cell slot differs from the previous
entry of the same wave range (each such entry costs the entry loop a register-image flush), and the
run-length distribution.  Usage: python scripts/tile_runs_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import ops  # noqa: E402

CHUNK = 2048


def main():
    cfg = bench.CONFIGS['p3d_fwdbwd']
    dev = torch.device('cuda:0')
    nfi.configure(scene_range=cfg[0], white_background=cfg[1], fine_sampling=True)
    batch = bench.make_inputs(cfg, dev, 0)
    ops.DEBUG_BACKWARD = {}
    bench.run_step(nfi, batch, cfg, True)
    torch.cuda.synchronize()
    ws = ops.DEBUG_BACKWARD['workspace'].cpu().numpy()
    B, H, S, R = 8, 128, 64, 256
    nsamp = B * H * H * 2 * S
    nx, ny = (R - 2) // 7 + 1, (R - 2) // 4 + 1
    K = B * 3 * nx * ny
    off = 0

    def take(nbytes):
        nonlocal off
        q = off
        off += (nbytes + 255) // 256 * 256
        return q
    take(nsamp * 32 * 4); take(nsamp * 4); take(nsamp * 4)
    take(K * 4); take(K * 4)
    o_off = take((K + 1) * 4)
    take((K + 1) * 4); take(16); take((K // 1024 + 1) * 8); take((3 * nsamp // CHUNK + K + 1) * 4)
    l_off = take((3 * nsamp + 128) * 16)
    offsets = ws[o_off:o_off + (K + 1) * 4].view(np.int32)
    total = int(offsets[K])
    rec = ws[l_off:l_off + total * 16].view(np.int32).reshape(total, 4)
    slot = rec[:, 1] & 31
    changes = 0
    n = 0
    runs = []
    for k in range(K):
        a, b = int(offsets[k]), int(offsets[k + 1])
        for c0 in range(a, b, CHUNK):
            c1 = min(b, c0 + CHUNK)
            per = (((c1 - c0) + 3) // 4 + 7) & ~7
            for w in range(4):
                w0, w1 = c0 + w * per, min(c1, c0 + (w + 1) * per)
                if w1 <= w0:
                    continue
                s = slot[w0:w1]
                ch = np.flatnonzero(s[1:] != s[:-1])
                changes += len(ch) + 1
                n += w1 - w0
                edges = np.concatenate([[0], ch + 1, [w1 - w0]])
                runs.append(np.diff(edges))
    runs = np.concatenate(runs)
    print(f'entries {n} (list {total}), cell changes {changes}: {changes / n:.3f} per entry; '
          f'mean run {runs.mean():.2f}, run quantiles 50/90/99 {np.quantile(runs, [0.5, 0.9, 0.99]).tolist()}')


if __name__ == '__main__':
    main()
