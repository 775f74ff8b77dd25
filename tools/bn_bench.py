"""Micro-benchmark of the ewvit BatchNorm(+act) kernels on the step's BN shapes:
fwd (train: stats + finalize + apply) and bwd (reduce + finalize + dx) through the
C-ABI, each recorded ITERS times into a HIP graph; prints device time and the
algorithmic HBM rate (fwd 3 tensor passes, bwd 5).
Usage: python tools/bn_bench.py [--iters N]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))
sys.path.insert(0, os.path.join(REPO, 'tools'))
from conv_bench import graph_time  # noqa: E402

# name: (rows M, channels C, act, groups)
SHAPES = {
    's6_dw_silu': (3136, 1536, 2, 1),
    's5_dw_silu': (12544, 960, 2, 1),
    's4_silu': (12544, 512, 2, 1),
    's6_proj': (3136, 256, 0, 1),
    's5_proj': (12544, 160, 0, 1),
    's2_silu': (200704, 192, 2, 1),
    's1_silu': (802816, 24, 2, 1),
    'mwt_fusion': (2408448, 128, 1, 3),
    'mwt_sep': (2408448, 64, 1, 3),
    'mwt_ms': (802816, 128, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    from ewvit import _lib as L
    lib = L.load()
    dev = torch.device('cuda', 0)
    for name, (M, C, act, groups) in SHAPES.items():
        x = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        w = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev) * 0.1
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        mean = torch.empty(groups, C, device=dev)
        inv = torch.empty(groups, C, device=dev)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        ws = torch.empty(lib.ewvit_bn_workspace(M, C, groups) // 4, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)

        def fwd():
            L.call('ewvit_bn_fwd', L.ptr(x), L.ptr(y), L.BF16, M, C, L.ptr(w), L.ptr(b), L.ptr(rm), L.ptr(rv), 1,
                   0.1, 1e-5, act, L.ptr(mean), L.ptr(inv), groups, L.ptr(cnt), L.ptr(ws), L.stream(x))

        def bwd():
            L.call('ewvit_bn_bwd', L.ptr(dy), L.ptr(x), L.ptr(dx), L.BF16, M, C, L.ptr(w), L.ptr(b), L.ptr(mean),
                   L.ptr(inv), act, L.ptr(dg), L.ptr(db), 0, groups, L.ptr(ws), L.stream(x))
        fwd()
        tf = min(graph_time(fwd, a.iters) for _ in range(3))
        tb = min(graph_time(bwd, a.iters) for _ in range(3))
        nb = M * C * 2
        print(f'{name:12s} M={M:8d} C={C:5d} {nb / 1e6:7.1f} MB | fwd {tf:7.1f} us {3 * nb / tf / 1e3:6.0f} GB/s | '
              f'bwd {tb:7.1f} us {5 * nb / tb / 1e3:6.0f} GB/s', flush=True)


if __name__ == '__main__':
    main()
