"""The torch (non-ewvit) kernels of one eager bench step, counted by kernel name and by the
chain of CPU ops / autograd nodes that launched them (torch.profiler event parents) — which
module or Function a fill or copy comes from.  (tools/glue_sources.py lists them by shape.)"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'efficient-wavelet-vit_amd'))
import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    frames = bench.CONFIGS[config]['frames'] if 'frames' in bench.CONFIGS[config] else 64
    step = bench.build_step(dev, frames, 0, graph=False, config=config)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    cnt = collections.Counter()
    kc = collections.Counter()
    for e in prof.events():
        if e.device_type != torch.autograd.DeviceType.CPU:
            continue
        for k in (e.kernels or []):
            kc[k.name[:90]] += 1
            if 'ewvit' in k.name:
                continue
            chain, q = [], e
            while q is not None and len(chain) < 8:
                chain.append(q.name[:60])
                q = q.cpu_parent
            cnt[(k.name[:60], ' < '.join(chain))] += 1
    print('--- device kernels in one eager step (non-ewvit first)')
    for n, c in kc.most_common():
        if 'ewvit' not in n:
            print(f'{c:4d}  {n}')
    print('--- glue kernels by CPU op chain')
    for (n, s), c in cnt.most_common(80):
        print(f'{c:4d}  {n:60s} | {s}')


if __name__ == '__main__':
    main()
