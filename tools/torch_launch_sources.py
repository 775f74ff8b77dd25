"""Where do the non-ewvit (torch / library) launches of a training step come from?
Runs one eager bench step under torch.profiler with Python stacks and prints, per
aten op that launched device work, its count and the innermost repo frames.
Usage: python tools/torch_launch_sources.py [--top 25]"""
import argparse
import collections
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--top', type=int, default=25)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    step = bench.build_step(dev, 64, 0, graph=False)
    for _ in range(2):
        step._eager()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
        step._eager()
        torch.cuda.synchronize()
    agg = collections.Counter()
    where = collections.defaultdict(collections.Counter)
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith('aten::'):
            continue
        if not ev.kernels:
            continue
        agg[ev.name] += len(ev.kernels)
        frames = [f for f in (ev.stack or []) if 'efficient-wavelet-vit_amd' in f or 'bench.py' in f]
        key = ' <- '.join(frames[:2]) if frames else 'shapes ' + str(ev.input_shapes)[:150]
        where[ev.name][key] += 1
    for name, n in agg.most_common(a.top):
        print(f'{n:5d}  {name}')
        for w, m in where[name].most_common(8):
            print(f'         {m:4d}  {w[:200]}')


if __name__ == '__main__':
    main()
