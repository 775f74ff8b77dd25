"""Micro-benchmark of the ewvit conv kernels on the step's conv shapes (HIP-event
timed, TFLOP/s per shape) — run under rocprofv3 --pmc for counter studies.
Usage: python tools/conv_bench.py [--iters N] [--only NAME]"""
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
    'bb_s5_expand': (64, 160, 14, 14, 960, 1, 1, 1),
    'bb_s5_project': (64, 960, 14, 14, 160, 1, 1, 1),
    'bb_head': (64, 256, 7, 7, 1280, 1, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--only', default=None)
    a = ap.parse_args()
    import ewvit
    dev = torch.device('cuda', 0)
    for name, (N, Cin, H, W, Cout, k, s, lv) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        x = torch.randn(N * lv, Cin, H, W, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w = (torch.randn(Cout, Cin * lv, k, k, device=dev) / (k * k * Cin * lv) ** 0.5).requires_grad_(True)
        b = torch.zeros(Cout, device=dev, requires_grad=True)
        y = ewvit.conv2d(x, w, b, s, lv)
        dy = torch.randn_like(y)
        flops = 2.0 * y.numel() * Cin * lv * k * k
        res = {}
        for phase in ('fwd', 'fwd+bwd'):
            for _ in range(3):
                y = ewvit.conv2d(x, w, b, s, lv)
                if phase != 'fwd':
                    y.backward(dy)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                y = ewvit.conv2d(x, w, b, s, lv)
                if phase != 'fwd':
                    y.backward(dy)
            e1.record()
            torch.cuda.synchronize()
            res[phase] = e0.elapsed_time(e1) / a.iters
        fl_all = flops * (3 if s == 1 else 6)   # stride-2 dgrad runs the full dense tap set
        print(f'{name:16s} fwd {res["fwd"] * 1e3:8.1f} us {flops / res["fwd"] / 1e9:7.1f} TF/s | '
              f'fwd+bwd {res["fwd+bwd"] * 1e3:8.1f} us ({fl_all / res["fwd+bwd"] / 1e9:7.1f} TF/s incl. packs)',
              flush=True)


if __name__ == '__main__':
    main()
