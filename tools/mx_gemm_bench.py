"""Times the config-5 module-path GEMMs (patch_to_embedding fwd / dgrad / wgrad, feat_map) on
ewvit_gemm_mx8 against the bf16 path (ewvit_gemm / the tall-K kernel): events around 20
back-to-back calls after a warm-up.  python tools/mx_gemm_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'efficient-wavelet-vit_amd'))
import ewvit  # noqa: E402

DEV = 'cuda'


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    g = torch.Generator(device=DEV).manual_seed(0)
    M, K, N = 64, 62720, 512
    X = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    G = torch.randn(M, N, device=DEV, generator=g)
    y = torch.empty(M, N, device=DEV)
    dx = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    dw = torch.empty(N, K, device=DEV)
    Xf = torch.randn(M, 512, device=DEV, generator=g)
    Wf = torch.randn(128, 512, device=DEV, generator=g)
    yf = torch.empty(M, 128, device=DEV)
    for fp8 in (False, True):
        r = {
            'pe fwd': t(lambda: ewvit.mm_nt(X, W, y, fp8=fp8)),
            'pe dgrad': t(lambda: ewvit.mm_nn(G, W, dx, fp8=fp8)),
            'pe wgrad': t(lambda: ewvit.mm_tn(G, X, dw, fp8=fp8)),
            'feat fwd': t(lambda: ewvit.mm_nt(Xf, Wf, yf, fp8=fp8)),
        }
        print('fp8' if fp8 else 'bf16', {k: round(v, 1) for k, v in r.items()}, flush=True)


if __name__ == '__main__':
    main()
