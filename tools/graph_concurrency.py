"""Do independent branches of a captured HIP graph run concurrently on this stack?
Captures K small kernels (a) on one stream, (b) split over two forked/joined streams,
(c) the same split but with one branch of large kernels, and times graph replay.
Usage: python tools/graph_concurrency.py [--k 200]"""
import argparse

import torch


def timed(g, iters=20):
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--k', type=int, default=200)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    small = [torch.zeros(64 * 1024, device=dev) for _ in range(4)]     # 256 KB: a few workgroups
    big = [torch.zeros(32 << 20, device=dev) for _ in range(2)]       # 128 MB
    side = torch.cuda.Stream()

    def chain(ts, n):
        for i in range(n):
            ts[i % len(ts)].add_(1.0)

    res = {}
    for name in ('serial_small', 'two_streams_small', 'serial_mixed', 'two_streams_mixed'):
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            chain(small, 2)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=cap):
                if name == 'serial_small':
                    chain(small[:2], a.k)
                    chain(small[2:], a.k)
                elif name == 'two_streams_small':
                    side.wait_stream(cap)
                    with torch.cuda.stream(side):
                        chain(small[2:], a.k)
                    chain(small[:2], a.k)
                    cap.wait_stream(side)
                elif name == 'serial_mixed':
                    chain(big, 8)
                    chain(small, a.k)
                else:
                    side.wait_stream(cap)
                    with torch.cuda.stream(side):
                        chain(small, a.k)
                    chain(big, 8)
                    cap.wait_stream(side)
        torch.cuda.current_stream().wait_stream(cap)
        res[name] = timed(g)
        print(f'{name:20s} {res[name]:9.1f} us', flush=True)


if __name__ == '__main__':
    main()
