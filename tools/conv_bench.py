"""Micro-benchmark of the ewvit conv kernels on the step's conv shapes.  Each phase
(fwd, fwd+bwd) is recorded ITERS times into a HIP graph and replayed, so the
numbers are device time without Python launch overhead.  --mm also times the
1x1 shapes as plain library GEMMs (torch.mm -> hipBLASLt) for comparison.
Usage: python tools/conv_bench.py [--iters N] [--only NAME] [--mm]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))

# name: (N, Cin, H, W, Cout, k, stride, levels)
SHAPES = {
    'mwt_fusion': (192, 56, 112, 112, 128, 3, 1, 1),
    'mwt_multiscale': (64, 128, 112, 112, 128, 3, 1, 3),
    'mwt_freq_conv': (64, 128, 112, 112, 128, 3, 2, 1),
    'bb_s2_fused': (64, 48, 56, 56, 192, 3, 1, 1),
    'bb_s4_expand': (64, 128, 28, 28, 512, 1, 1, 1),
    'bb_s5_expand': (64, 160, 14, 14, 960, 1, 1, 1),
    'bb_s5_project': (64, 960, 14, 14, 160, 1, 1, 1),
    'bb_s6_expand': (64, 256, 7, 7, 1536, 1, 1, 1),
    'bb_head': (64, 256, 7, 7, 1280, 1, 1, 1),
}


def graph_time(fn, iters):
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
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3     # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--only', default=None)
    ap.add_argument('--mm', action='store_true')
    a = ap.parse_args()
    import ewvit
    dev = torch.device('cuda', 0)
    for name, (N, Cin, H, W, Cout, k, s, lv) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        x = torch.randn(N * lv, Cin, H, W, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w = (torch.randn(Cout, Cin * lv, k, k, device=dev) / (k * k * Cin * lv) ** 0.5).requires_grad_(True)
        y = ewvit.conv2d(x, w, None, s, lv)
        dy = torch.randn_like(y)
        flops = 2.0 * y.numel() * Cin * lv * k * k

        def fwd():
            ewvit.conv2d(x, w, None, s, lv)

        def fwdbwd():
            x.grad = None
            w.grad = None
            ewvit.conv2d(x, w, None, s, lv).backward(dy)
        tf = graph_time(fwd, a.iters)
        tb = graph_time(fwdbwd, a.iters)
        fl_all = flops * (3 if s == 1 else 6)   # stride-2 dgrad runs the full dense tap set
        line = (f'{name:16s} fwd {tf:8.1f} us {flops / tf / 1e6:7.1f} TF/s | fwd+bwd {tb:8.1f} us '
                f'({fl_all / tb / 1e6:7.1f} TF/s incl. packs)')
        if a.mm and k == 1 and s == 1:
            M = N * H * W
            x2 = torch.randn(M, Cin, device=dev, dtype=torch.bfloat16)
            w2 = torch.randn(Cout, Cin, device=dev, dtype=torch.bfloat16)
            d2 = torch.randn(M, Cout, device=dev, dtype=torch.bfloat16)
            t1 = graph_time(lambda: torch.mm(x2, w2.t()), a.iters)
            t2 = graph_time(lambda: torch.mm(d2, w2), a.iters)
            t3 = graph_time(lambda: torch.mm(d2.t(), x2), a.iters)
            line += f' || hipBLASLt fwd {t1:6.1f} dgrad {t2:6.1f} wgrad {t3:6.1f} us'
        print(line, flush=True)


if __name__ == '__main__':
    main()
