"""Where the torch copies and fills of one eager bench step come from: the step of bench.py
(config 2) run eagerly under torch.profiler (CPU ops with Python stacks), aten::copy_ /
fill_ / zero_ calls grouped by the innermost repo frame that issued them.
Usage (GPU): python tools/glue_sources.py"""
import collections
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))
import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    step = bench.build_step(dev, 64, 0, graph=False, config=2)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    want = ('aten::copy_', 'aten::fill_', 'aten::zero_', 'aten::zeros', 'aten::zeros_like', 'aten::cat',
            'aten::contiguous', 'aten::clone')
    by = collections.Counter()
    for ev in prof.events():
        if ev.name not in want:
            continue
        frames = [f for f in (ev.stack or []) if ('/network/' in f or '/ewvit/' in f or 'bench.py' in f)
                  and 'glue_sources' not in f]
        site = frames[0] if frames else '(no repo frame)'
        shp = str(ev.input_shapes)[:80]
        if '[0]' in shp:
            continue                             # zero-element tensors: no kernel
        by[(ev.name, site, shp)] += 1
    for (name, site, shp), n in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f'{n:4d} {name:18s} {site}  {shp}')


if __name__ == '__main__':
    main()
