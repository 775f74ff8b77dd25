"""Time the BatchNorm(+SiLU) kernels at the backbone's shapes (config 2: 64 frames) over
back-to-back launches replayed from a HIP graph: ewvit_bn_fwd (stats + apply) and
ewvit_bn_bwd (reduce + dx).  Prints us per call and the effective HBM rate of the
minimum traffic (fwd: read x, read x + write y = 3 tensor passes; bwd: read
x and dy twice + write dx = 5 passes)."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'efficient-wavelet-vit_amd')]
from ewvit import _lib as L  # noqa: E402

SHAPES = [(3136, 1536, 2), (3136, 256, 0), (12544, 960, 2), (12544, 512, 2), (12544, 160, 0), (50176, 256, 2),
          (200704, 192, 2), (802816, 24, 2)]


def timeit(fn, n=20, reps=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (n * reps) * 1e3


def main():
    lib = L.load()
    for M, C, act in SHAPES:
        x = torch.randn(M, C, device='cuda').bfloat16()
        dy = torch.randn(M, C, device='cuda').bfloat16()
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        w = torch.rand(C, device='cuda') + 0.5
        b = torch.randn(C, device='cuda') * 0.1
        rm, rv = torch.zeros(C, device='cuda'), torch.ones(C, device='cuda')
        mean, inv = torch.empty(C, device='cuda'), torch.empty(C, device='cuda')
        dg, db = torch.empty(C, device='cuda'), torch.empty(C, device='cuda')
        ws = torch.empty(lib.ewvit_bn_workspace(M, C, 1) // 4, device='cuda')
        cnt = torch.zeros((), dtype=torch.int64, device='cuda')
        bf = 1

        def fwd():
            L.call('ewvit_bn_fwd', L.ptr(x), L.ptr(y), bf, M, C, L.ptr(w), L.ptr(b), L.ptr(rm), L.ptr(rv), 1, 0.01,
                   1e-3, act, L.ptr(mean), L.ptr(inv), 1, L.ptr(cnt), L.ptr(ws), L.stream(y))

        def bwd():
            L.call('ewvit_bn_bwd', L.ptr(dy), L.ptr(x), L.ptr(dx), bf, M, C, L.ptr(w), L.ptr(b), L.ptr(mean),
                   L.ptr(inv), act, L.ptr(dg), L.ptr(db), 0, 1, L.ptr(ws), L.stream(dx))
        fwd()
        tf, tb = timeit(fwd), timeit(bwd)
        mb = M * C * 2 / 1e6
        print(f'[{M:6d} x {C:4d}] act {act}: fwd {tf:6.1f} us ({3 * mb / tf * 1e-3:5.2f} TB/s of 3 passes)   '
              f'bwd {tb:6.1f} us ({5 * mb / tb * 1e-3:5.2f} TB/s of 5 passes)   tensor {mb:.1f} MB', flush=True)


if __name__ == '__main__':
    main()
