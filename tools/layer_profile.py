"""Per-launch attribution of the bench step's ewvit kernels: the eager step is run
with HIP events around every C-ABI launch; launches are grouped by (entry point,
integer arguments = shape) and printed by total time, plus the event-bracketed
total of the whole step (ewvit + torch kernels).
Usage: python tools/layer_profile.py [--top N]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--top', type=int, default=60)
    a = ap.parse_args()
    import ewvit
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    step = bench.build_step(dev, 64, 0)
    for _ in range(3):
        step._eager()
    torch.cuda.synchronize()
    ewvit._lib.enable_timing(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    step._eager()
    e1.record()
    torch.cuda.synchronize()
    det = ewvit._lib.timing_detail()
    ewvit._lib.enable_timing(False)
    agg = {}
    tot = 0.0
    for name, ints, s, e, _ in det:
        t = s.elapsed_time(e) * 1e3
        tot += t
        k = (name, ints)
        c, u = agg.get(k, (0, 0.0))
        agg[k] = (c + 1, u + t)
    print(f'step (events, eager): {e0.elapsed_time(e1):.2f} ms; ewvit launches {len(det)}, {tot / 1e3:.2f} ms')
    byname = {}
    for (n, _), (c, u) in agg.items():
        byname[n] = byname.get(n, 0.0) + u
    for n, u in sorted(byname.items(), key=lambda x: -x[1]):
        print(f'  {n:32s} {u / 1e3:7.3f} ms')
    print()
    for (n, ints), (c, u) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f'{u:9.1f} us {c:3d}x  {n:28s} {ints}')


if __name__ == '__main__':
    main()
