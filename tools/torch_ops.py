"""Which torch (non-ewvit) ops of the bench step launch GPU kernels, and from where:
the eager step under torch.profiler with Python stacks, aten ops grouped by
(name, top user frame).  Usage: python tools/torch_ops.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))

import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    step = bench.build_step(dev, 64, 0, graph=False)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    rows = {}
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CPU and ev.name.startswith('aten::') and ev.device_time_total > 0:
            frames = [f for f in (ev.stack or []) if ('wavelet' in f or 'bench.py' in f) and 'torch_ops.py' not in f]
            key = (ev.name, frames[0] if frames else '?')
            c, t = rows.get(key, (0, 0.0))
            rows[key] = (c + 1, t + ev.self_device_time_total)
    for (n, f), (c, t) in sorted(rows.items(), key=lambda x: -x[1][0])[:60]:
        print(f'{c:4d} {t:9.1f} us  {n:28s} {f[-90:]}')


if __name__ == '__main__':
    main()
