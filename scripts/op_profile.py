"""torch.profiler op table of the eager inversion step (GPU box): which aten ops launch the ~280
generic elementwise / fill kernels per vgg step (B=4), with their Python call sites.
Usage: python scripts/op_profile.py [loss] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'nerf-from-image_amd'), os.path.join(ROOT, 'scripts')]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402
from nfi import inversion, lpips, producer  # noqa: E402


def main():
    loss = sys.argv[1] if len(sys.argv) > 1 else 'vgg'
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
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
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False,
                 experimental_config=torch._C._profiler._ExperimentalConfig(verbose=True)) as prof:
        inversion.invert(gen, target, batch['cam'], batch['focal'], w_avg, icfg, lpips_net=net)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by='count', row_limit=45, max_name_column_width=40))
    # call sites: the innermost nfi / torch.nn frames of every top-level aten op that launches work
    import collections
    sites = collections.Counter()
    for e in prof.events():
        if not e.name.startswith('aten::') or e.name in ('aten::empty', 'aten::view', 'aten::as_strided', 'aten::detach',
                                                          'aten::reshape', 'aten::select', 'aten::transpose', 'aten::unsqueeze',
                                                          'aten::slice', 'aten::expand', 'aten::empty_like', 'aten::empty_strided',
                                                          'aten::permute', 'aten::narrow', 'aten::t', 'aten::mT', 'aten::_reshape_alias',
                                                          'aten::_unsafe_view', 'aten::result_type'):
            continue
        fr = [f for f in (e.stack or []) if 'nfi/' in f or 'nn/modules' in f or 'autograd' in f]
        if e.cpu_parent is not None and e.cpu_parent.name.startswith('aten::'):
            continue
        sites[(e.name, ' <- '.join(f.split('nfi/')[-1] for f in fr[:3]))] += 1
    ex = [e for e in prof.events() if e.name == 'aten::mul'][:1]
    print('sample stack:', ex[0].stack if ex else None)
    for (n, st), c in sites.most_common(70):
        print(f'{c / steps:6.1f}/step  {n:24s} {st}')


if __name__ == '__main__':
    main()
