"""Eager conv fwd/bwd on the bench shapes, synchronising and printing after each
pass (locates a failing kernel/shape).  Usage: python tools/conv_debug.py [glds]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))
sys.path.insert(0, os.path.join(REPO, 'tools'))
from conv_bench import SHAPES  # noqa: E402


def main():
    import ewvit
    lib = ewvit._lib.load()
    lib.ewvit_conv2d_set_glds(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    dev = torch.device('cuda', 0)
    for name, (N, Cin, H, W, Cout, k, s, lv) in SHAPES.items():
        x = torch.randn(N * lv, Cin, H, W, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w = (torch.randn(Cout, Cin * lv, k, k, device=dev) / (k * k * Cin * lv) ** 0.5).requires_grad_(True)
        print(name, 'fwd', flush=True)
        y = ewvit.conv2d(x, w, None, s, lv)
        torch.cuda.synchronize()
        print(name, 'bwd', flush=True)
        y.backward(torch.randn_like(y))
        torch.cuda.synchronize()
        print(name, 'ok', float(x.grad.float().abs().mean()), float(w.grad.abs().mean()), flush=True)


if __name__ == '__main__':
    main()
