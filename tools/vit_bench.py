"""Micro-benchmark of the ViT encoder (sfe.Transformer, depth 2, 64 frames = 128 rows) fwd + bwd:
the fused layer (csrc/vit.hip) against the module path, each replayed from a HIP graph.
Run under rocprofv3 --kernel-trace --stats for per-kernel times.
Usage: python tools/vit_bench.py [--iters 20] [--frames 64]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--frames', type=int, default=64)
    args = ap.parse_args()
    from network.sfe import Transformer
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    m = Transformer(512, 2, 8, 64, 2048, 0.15).to(dev).train()
    x = torch.randn(args.frames, 2, 512, device=dev, requires_grad=True)
    w = torch.randn(args.frames, 2, 512, device=dev)
    out = {}
    for mode in os.environ.get('VIT_BENCH_MODES', '1,0').split(','):
        os.environ['EWVIT_VIT_FUSED'] = mode

        def step():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                y = m(x)
            (y * w).sum().backward()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step()
        torch.cuda.current_stream().wait_stream(s)
        for p in m.parameters():
            p.grad = None
        x.grad = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out['fused' if mode == '1' else 'module'] = round(e0.elapsed_time(e1) / args.iters * 1e3, 1)
    print({'vit_fwd_bwd_us': out, 'frames': args.frames})


if __name__ == '__main__':
    main()
