"""Isolated timing of the MWT front end (the fused ewvit_dwt_hf_upsample_fused, and the
two-launch ewvit_dwt_haar_fwd + ewvit_hf_upsample it replaces) at the bench shape
(config 2: 64 x 3 x 224^2 fp32 frames, 3 levels, bf16 bands): ITERS back-to-back launches captured in one HIP graph, timed by events around the replay,
so the per-launch figure is the kernel duration (as rocprofv3 reports it) without
the per-launch event gaps of bench.py's eager pass.

  python tools/dwt_bench.py [--n 64] [--hw 224] [--levels 3] [--iters 50]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


def graph_us(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float('inf')
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def measure(n=64, hw=224, levels=3, iters=50, channels=None):
    """-> {'dwt_us', 'dwt_bytes', 'up_us', 'up_bytes', 'fused_us', 'fused_bytes', 'channels'}
    (algorithmic bytes per launch) for the hf_conv input layout the MWT writes: `channels` = 9
    (the real band channels, ewvit.hfsep.HF9) or 16 (zero-padded); default: the MWT's own."""
    from ewvit import hfsep, ops
    if channels is None:
        channels = 9 if hfsep.HF9 else 16
    dev = torch.device('cuda', 0)
    x = torch.randn(n, 3, hw, hw, device=dev)
    ll, yh, sizes = ops._dwt_flat(x, levels, torch.bfloat16)
    dwt_bytes = x.numel() * 4 + (yh.numel() + ll.numel()) * 2
    dwt_us = graph_us(lambda: ops._dwt_flat(x, levels, torch.bfloat16), iters)
    c = channels
    out = ops.hf_upsample(yh, n, 3, hw, hw, levels, (hw // 2, hw // 2), torch.bfloat16, c)
    up_bytes = yh.numel() * 2 + out.numel() * 2
    up_us = graph_us(lambda: ops.hf_upsample(yh, n, 3, hw, hw, levels, (hw // 2, hw // 2), torch.bfloat16, c),
                     iters)
    fused_us = fused_bytes = None                      # the fused launch takes W <= 224
    if ops.L.load().ewvit_dwt_hf_fused_ok(n, 3, hw, hw, levels, hw // 2, hw // 2, c):
        fused_us = graph_us(lambda: ops._dwt_hf_fused_op(x, levels, torch.bfloat16, c), iters)
        fused_bytes = x.numel() * 4 + out.numel() * 2  # frames in + hf_conv input out
    return {'dwt_us': dwt_us, 'dwt_bytes': dwt_bytes, 'up_us': up_us, 'up_bytes': up_bytes,
            'fused_us': fused_us, 'fused_bytes': fused_bytes, 'channels': c}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=64)
    ap.add_argument('--hw', type=int, default=224)
    ap.add_argument('--levels', type=int, default=3)
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--channels', type=int, nargs='*', default=[9, 16])
    a = ap.parse_args()
    for ch in a.channels:
        r = measure(a.n, a.hw, a.levels, a.iters, ch)
        for k in ('dwt', 'up', 'fused'):
            us, b = r[k + '_us'], r[k + '_bytes']
            if us is None:
                continue
            print(f'{ch:2d}ch {k:5s} {us:8.2f} us  {b / 1e6:7.2f} MB  {b / us / 1e3:7.1f} GB/s', flush=True)


if __name__ == '__main__':
    main()
