"""Per-launch floor of back-to-back kernels in a HIP graph (the fixed cost every small kernel
of the step pays): graph-replayed chains of tiny torch fills and of ewvit's weight-gradient
reduce kernel on a 1-element problem, microseconds per launch.
Usage: python tools/launch_floor.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))
sys.path.insert(0, os.path.join(REPO, 'tools'))


def main():
    from conv_bench import graph_time
    dev = torch.device('cuda', 0)
    for n in (1024, 1 << 20, 16 << 20):
        t = torch.empty(n // 4, device=dev)
        print(f'fill {n:>9d} B: {graph_time(lambda: t.fill_(1.0), 50):7.2f} us/launch', flush=True)
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    lib = L.load()
    for (N, H, W, Cin, Cout) in ((1, 8, 8, 8, 8), (64, 7, 7, 256, 1536)):
        x = torch.randn(N, Cin, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, Cout, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dw = torch.empty(Cout, Cin, 1, 1, device=dev)
        ws = torch.empty(int(lib.ewvit_conv2d_bwd_weight_workspace(N, H, W, Cin, Cout, 1, 1)) // 4 + 64, device=dev)

        def wg():
            L.call('ewvit_conv2d_bwd_weight', L.ptr(x), L.ptr(dy), L.ptr(dw), None, 0, N, H, W, Cin, Cout, 1, 1, 0, 0,
                   Cin, dw.stride(0), dw.stride(1), dw.stride(3), L.ptr(ws), L.stream(dw))
        print(f'wgrad 1x1 {N}x{H}x{W} {Cin}->{Cout}: {graph_time(wg, 50):7.2f} us/call', flush=True)


if __name__ == '__main__':
    main()
