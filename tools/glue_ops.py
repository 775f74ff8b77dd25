"""Diagnostic (GPU): which torch ops launch the non-ewvit ("glue") kernels of the config-2
training step — one eager step under torch.profiler after warm-up; prints the aten ops that
launched fill / copy / elementwise kernels with their call counts and the Python call sites
(innermost frames in the repo, or the op's input shapes
when the profiler records no Python stack).  Output: stdout + gpurun_out/glue_ops.txt."""
import collections
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'efficient-wavelet-vit_amd')]
import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    step = bench.build_step(dev, 64, 0, graph=False)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    # kernel -> its launching aten op (the innermost CPU op enclosing the launch) + repo stack
    evs = prof.events()
    by_site = collections.Counter()
    kern_us = collections.Counter()
    for e in evs:
        if e.device_type != torch.autograd.DeviceType.CPU or not e.kernels:
            continue
        if not e.name.startswith('aten::'):
            continue
        stack = [s for s in (e.stack or []) if ('efficient-wavelet-vit_amd' in s or 'bench.py' in s)
                 and 'torch/' not in s]
        site = ' <- '.join(s.split('/')[-1] for s in stack[:3]) or str(e.input_shapes)[:90]
        for k in e.kernels:
            if 'ewvit' in k.name:
                continue
            by_site[(e.name, k.name[:60], site)] += 1
            kern_us[(e.name, k.name[:60], site)] += k.duration
    lines = []
    for key, n in by_site.most_common(80):
        lines.append(f'{n:4d} x {kern_us[key] / max(n, 1):6.1f} us  {key[0]:28s} {key[1]:60s} {key[2]}')
    out = '\n'.join(lines)
    print(out, flush=True)
    os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
    open(os.path.join(REPO, 'gpurun_out', 'glue_ops.txt'), 'w').write(out + '\n')


if __name__ == '__main__':
    main()
