import os, sys
sys.path.insert(0, '/root/repo/nerf-from-image_amd'); sys.path.insert(0, '/root/repo')
import torch, bench, nfi
from nfi import ops
stash = {}
orig = torch.empty
cfg = bench.CONFIGS['p3d_fwdbwd']
dev = torch.device('cuda:0')
batch = bench.make_inputs(cfg, dev, 0)
# capture tile_counts via save_for_backward hook
orig_save = torch.autograd.function.FunctionCtx.save_for_backward
def save(ctx, *t):
    stash['tc'] = t[-1]
    return orig_save(ctx, *t)
torch.autograd.function.FunctionCtx.save_for_backward = save
bench.run_step(nfi, batch, cfg, True)
torch.cuda.synchronize()
tc = stash['tc'].long().cpu()
E = int(tc.sum()); nz = int((tc > 0).sum())
chunks = int(((tc + 2047) // 2048).sum())
print('tiles', tc.numel(), 'nonempty', nz, 'entries', E, 'chunks', chunks, 'entries/sample', E / (8*128*128*128))
q = torch.quantile(tc[tc > 0].double(), torch.tensor([0.1, 0.5, 0.9, 0.99], dtype=torch.double))
print('count quantiles (nonempty)', q.tolist(), 'max', int(tc.max()))
