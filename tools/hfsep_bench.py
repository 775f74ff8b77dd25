"""Isolated timing of the MWT seperate conv at the bench shape (config 2: 3 levels x 64 frames
at 112^2, 16 HF channels in, 64 out): the grouped csrc/hfsep.hip kernels (forward with the
BatchNorm partial statistics; weight gradient + reduce) against the block-diagonal dense
conv they replaced (ewvit.conv2d forward; its weight gradient), each as ITERS back-to-back
launches replayed from one HIP graph, uncapped and under the MWT's grid cap.

  python tools/hfsep_bench.py [--n 64] [--hw 112] [--iters 20] [--cap 160]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))
sys.path.insert(0, os.path.join(REPO, 'tools'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=64)
    ap.add_argument('--hw', type=int, default=112)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--cap', type=int, default=160)
    args = ap.parse_args()
    import ewvit
    from ewvit import _lib as L
    from dwt_bench import graph_us
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    convs = [torch.nn.Conv2d(3, 18, 3, padding=1).to(dev) for _ in range(3)]
    Lv, N, H = 3, args.n, args.hw
    x = torch.zeros(Lv * N, H, H, 16, device=dev, dtype=torch.bfloat16)
    x[..., :9] = torch.randn(Lv * N, H, H, 9, device=dev).to(torch.bfloat16)
    x = x.permute(0, 3, 1, 2)
    x9 = x[:, :9].contiguous(memory_format=torch.channels_last)     # the 9 real band channels only
    shift = torch.zeros(64, device=dev)
    dy = torch.randn(Lv * N, 64, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    npx = Lv * N * H * H
    ws = torch.empty(int(L.load().ewvit_hfsep_bwd_weight_workspace(Lv * N, H, H)) // 4 + 1, device=dev)
    out = {}

    def run(tag, cap, xs=16):
        xin = x if xs == 16 else x9
        with L.grid_cap(cap), L.launch_cap(cap):
            nparts = int(L.load().ewvit_hfsep_fwd_parts(Lv, N, H, H))
            part = torch.empty(Lv, nparts, 128, device=dev)
            shifts = torch.empty(Lv, 64, device=dev)
            y = torch.empty(Lv * N, 64, H, H, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
            wsz = int(L.load().ewvit_hfsep_bwd_weight_workspace(Lv * N, H, H)) // 4 + 1
            wsp = ws if ws.numel() >= wsz else torch.empty(wsz, device=dev)
            dws = [torch.empty(18, 3, 3, 3, device=dev) for _ in range(3)]
            dbs = [torch.empty(18, device=dev) for _ in range(3)]
            prm = [c.weight.detach() for c in convs] + [c.bias.detach() for c in convs]

            def fwd():
                L.call('ewvit_hfsep_fwd', L.ptr(xin), L.ptr(y), Lv, N, H, H, xs, *[L.ptr(t) for t in prm], L.ptr(shift),
                       L.ptr(part), L.ptr(shifts), nparts, L.stream(y))

            def wg():
                L.call('ewvit_hfsep_bwd_weight', L.ptr(xin), L.ptr(dy), Lv * N, H, H, xs, *[L.ptr(t) for t in dws + dbs],
                       L.ptr(wsp), L.stream(dy))
            f_us, w_us = graph_us(fwd, args.iters), graph_us(wg, args.iters)
        out[tag] = {'fwd_us': round(f_us, 2), 'wgrad_us': round(w_us, 2),
                    'fwd_GBs': round(npx * (2 * xs + 128) / f_us / 1e3, 1),
                    'wgrad_GBs': round(npx * (128 + 2 * xs) / w_us / 1e3, 1)}

    run('grouped', 0)
    run(f'grouped_cap{args.cap}', args.cap)
    run('grouped_x9', 0, 9)
    run(f'grouped_x9_cap{args.cap}', args.cap, 9)
    # the block-diagonal dense conv it replaced (16 -> 64 on the MFMA conv kernels)
    w = torch.cat([torch.nn.functional.pad(c.weight.detach(), (0, 0, 0, 0, i * 3, 13 - 3 * i)) for i, c in enumerate(convs)])
    w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, 0, 0, 10)).contiguous()
    b = torch.zeros(64, device=dev)
    xc = x.contiguous(memory_format=torch.channels_last)
    for tag, cap in (('dense', 0), (f'dense_cap{args.cap}', args.cap)):
        with L.grid_cap(cap), L.launch_cap(cap):
            wp, _ = ewvit.conv._pack(w, 16, True, False)
            yd = torch.empty(Lv * N, 64, H, H, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
            wsb = L.load().ewvit_conv2d_bwd_weight_workspace(Lv * N, H, H, 16, 64, 3, 1)
            wsd = torch.empty(wsb // 4 + 1, device=dev)
            dw = torch.empty(64, 16, 3, 3, device=dev)
            db = torch.empty(64, device=dev)

            def dfwd():
                L.call('ewvit_conv2d_fwd', L.ptr(xc), L.ptr(wp), L.ptr(b), L.ptr(yd), Lv * N, H, H, 16, 64, 3, 1, 0, 0,
                       L.stream(yd))

            def dwg():
                L.call('ewvit_conv2d_bwd_weight', L.ptr(xc), L.ptr(dy), L.ptr(dw), L.ptr(db), 0, Lv * N, H, H, 16, 64,
                       3, 1, 0, 0, 16, 144, 9, 1, L.ptr(wsd), L.stream(dw))
            out[tag] = {'fwd_us': round(graph_us(dfwd, args.iters), 2), 'wgrad_us': round(graph_us(dwg, args.iters), 2)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
