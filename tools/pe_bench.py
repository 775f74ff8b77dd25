"""patch_to_embedding GEMMs (sfe.py:155: [64, 62720] x [62720, 512]) on ewvit_gemm with
several split-K counts: forward (split-K + reduce) and input gradient, graph-replayed.
Usage: python tools/pe_bench.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


def t_graph(fn, iters=20):
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
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    import ewvit
    dev = torch.device('cuda', 0)
    M, K, N = 64, 62720, 512
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev) * 0.01
    wb = w.to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev)
    g = torch.randn(M, N, device=dev)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    out = {}
    for sk in (16, 32, 64, 128, 245):
        out[f'fwd_f32w_sk{sk}'] = round(t_graph(lambda: ewvit.mm_nt(x, w, y, bias=b, splitk=sk)), 1)
    for sk in (64, 128, 245):
        out[f'fwd_bf16w_sk{sk}'] = round(t_graph(lambda: ewvit.mm_nt(x, wb, y, bias=b, splitk=sk)), 1)
    out['fwd_tallk'] = round(t_graph(lambda: ewvit.mm_nt(x, w, y, bias=b)), 1)
    out['dgrad_f32w'] = round(t_graph(lambda: ewvit.mm_nn(g, w, dx)), 1)
    out['dgrad_bf16w'] = round(t_graph(lambda: ewvit.mm_nn(g, wb, dx)), 1)
    out['pack_w_bf16'] = round(t_graph(lambda: wb.copy_(w)), 1)
    print(out)


if __name__ == '__main__':
    main()
