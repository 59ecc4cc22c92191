"""Which lines of the package issue the ATen ops of one eager inversion step (forward and the
backward's python-side code): a TorchDispatchMode that counts every op by the innermost nfi
source line on the python stack.  Usage (GPU box): python scripts/op_sources.py [loss] [B]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import inversion, lpips, producer  # noqa: E402

SKIP = {'aten.empty.memory_format', 'aten.empty_strided.default', 'aten.view.default', 'aten.detach.default',
        'aten._to_copy.default', 'aten.t.default', 'aten.transpose.int', 'aten.select.int', 'aten.slice.Tensor',
        'aten.unsqueeze.default', 'aten.expand.default', 'aten.as_strided.default', 'aten._unsafe_view.default',
        'aten.permute.default', 'aten.squeeze.dim', 'aten.unbind.int', 'aten.split.Tensor', 'aten.alias.default',
        'aten.empty_like.default', 'aten.reshape.default', 'aten.lift_fresh.default', 'aten._reshape_alias.default'}


class Count(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name not in SKIP:
            where = '?'
            for fr in reversed(traceback.extract_stack()):
                if '/nfi/' in fr.filename or fr.filename.endswith('bench.py'):
                    where = f'{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}'
                    break
            if where == '?':        # backward: the forward line that created the running node
                node = torch._C._current_autograd_node()
                tb = None if node is None else node.metadata.get('traceback_')
                if tb:
                    lines = [ln for ln in ''.join(tb).split('\n') if '/nfi/' in ln]
                    if lines:
                        last = lines[-1].strip()
                        where = 'bwd ' + type(node).__name__ + ' <- ' + last.split('/nfi/')[-1]
                else:
                    where = 'bwd ' + (type(node).__name__ if node is not None else '?')
            self.c[(where, name)] += 1
        return func(*args, **(kwargs or {}))


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
    icfg = inversion.InversionConfig(steps=2, resolution=128, samples=64, loss=loss)
    inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
    torch.cuda.synchronize()
    icfg.steps = 3
    with torch.autograd.detect_anomaly(check_nan=False), Count() as m:
        inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
    torch.cuda.synchronize()
    tot = sum(m.c.values())
    print(f'{tot / icfg.steps:.0f} ops per step (3 steps incl. setup)')
    for (where, name), n in m.c.most_common(120):
        print(f'{n / icfg.steps:6.1f}  {name:40s} {where}')


if __name__ == '__main__':
    main()
