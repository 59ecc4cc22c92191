"""Do two half-batch renders on two HIP streams overlap?  The three big launches are bound by
different things (render_fwd / field_bwd: issue and gather latency; tile_kernel: HBM), so a
half batch's tile pass might run beside the other half's field backward.  Times one B=8
fwd+bwd step against two B=4 steps back to back and two B=4 steps on two streams (plain and
staggered by one forward).  Usage (GPU box): python scripts/stream_overlap_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nerf-from-image_amd'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import nfi  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device('cuda:0')
    cfg = bench.CONFIGS['p3d_fwdbwd']
    nfi.configure(scene_range=cfg[0], white_background=cfg[1], fine_sampling=True)
    half = cfg[:3] + (cfg[3] // 2,) + cfg[4:]
    full = bench.make_inputs(cfg, dev, 1)
    h1, h2 = bench.make_inputs(half, dev, 2), bench.make_inputs(half, dev, 3)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def step_full():
        bench.run_step(nfi, full, cfg, True)

    def step_seq():
        bench.run_step(nfi, h1, half, True)
        bench.run_step(nfi, h2, half, True)

    def step_two_streams(stagger):
        main = torch.cuda.current_stream(dev)
        s1.wait_stream(main)
        s2.wait_stream(main)
        with torch.cuda.stream(s1):
            bench.run_step(nfi, h1, half, True)
        if stagger:
            s2.wait_stream(s1)      # crude: the whole first half before the second starts
        with torch.cuda.stream(s2):
            bench.run_step(nfi, h2, half, True)
        main.wait_stream(s1)
        main.wait_stream(s2)

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    for _ in range(2):
        print(f'B=8 one stream        {timeit(step_full):6.3f} ms', flush=True)
        print(f'2x B=4 one stream     {timeit(step_seq):6.3f} ms', flush=True)
        print(f'2x B=4 two streams    {timeit(lambda: step_two_streams(False)):6.3f} ms', flush=True)


if __name__ == '__main__':
    main()
