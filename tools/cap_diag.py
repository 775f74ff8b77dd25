"""MWT forward/backward under a grid cap vs uncapped: per-parameter gradient error
(diagnosis of capped-walk differences; run with EWVIT_LIB to compare library builds)."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'efficient-wavelet-vit_amd')]
import ewvit  # noqa: E402
import network.mwt as mw  # noqa: E402

DEV = 'cuda'


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


def run(cap, hw=96, n=4, seed=5):
    torch.manual_seed(seed)
    m = mw.MWT(3, 128, 3).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(n, 3, hw, hw, device=DEV, generator=torch.Generator(DEV).manual_seed(1))
    with ewvit._lib.grid_cap(cap), torch.autocast('cuda', dtype=torch.bfloat16):
        y = m(x)
    dy = torch.randn(y.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(2))
    with ewvit._lib.grid_cap(cap):
        y.float().backward(dy)
    torch.cuda.synchronize()
    return y.detach().float(), {k: p.grad for k, p in m.named_parameters()}


for hw in (96, 64):
    y0, g0 = run(0, hw)
    yz, gz = run(0, hw)
    for cap in (16, 160):
        y1, g1 = run(cap, hw)
        print(f'hw={hw} cap={cap} out {rel(y1, y0):.2e} (repeat {rel(yz, y0):.2e})')
        for k in g0:
            if g0[k] is None:
                continue
            print(f'   {k:40s} {rel(g1[k], g0[k]):.2e}   repeat {rel(gz[k], g0[k]):.2e}')
