"""Micro-benchmark of the ewvit conv kernels on the step's conv shapes.  Each phase
(fwd, dgrad, wgrad: direct C-ABI calls, no autograd) is recorded ITERS times into a HIP graph and replayed, so the
numbers are device time without Python launch overhead.  --mm also times the
1x1 shapes as plain library GEMMs (torch.mm -> hipBLASLt) for comparison.
Usage: python tools/conv_bench.py [--iters N] [--only NAME] [--mm]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))

# name: (N, Cin, H, W, Cout, k, stride, levels)
SHAPES = {
    'mwt_fusion': (192, 64, 112, 112, 128, 3, 1, 1),
    'mwt_multiscale': (64, 128, 112, 112, 128, 3, 1, 3),
    'mwt_freq_conv': (64, 128, 112, 112, 128, 3, 2, 1),
    'bb_s2_fused': (64, 48, 56, 56, 192, 3, 1, 1),
    'bb_s1_fused': (64, 24, 112, 112, 24, 3, 1, 1),
    'mwt_seperate': (192, 16, 112, 112, 64, 3, 1, 1),
    'bb_s2_project': (64, 192, 56, 56, 48, 1, 1, 1),
    'bb_s2e_project': (64, 96, 56, 56, 48, 1, 1, 1),
    'bb_s3_fused': (64, 64, 28, 28, 256, 3, 1, 1),
    'bb_s3_project': (64, 256, 28, 28, 64, 1, 1, 1),
    'bb_s2_entry': (64, 24, 112, 112, 96, 3, 2, 1),
    'bb_s3_entry': (64, 48, 56, 56, 192, 3, 2, 1),
    'bb_s4_expand': (64, 128, 28, 28, 512, 1, 1, 1),
    'bb_s5_expand': (64, 160, 14, 14, 960, 1, 1, 1),
    'bb_s5_project': (64, 960, 14, 14, 160, 1, 1, 1),
    'bb_s6_expand': (64, 256, 7, 7, 1536, 1, 1, 1),
    'bb_s6_project': (64, 1536, 7, 7, 256, 1, 1, 1),
    'bb_head': (64, 256, 7, 7, 1280, 1, 1, 1),
}


EAGER = False


def graph_time(fn, iters):
    if EAGER:                      # plain launches (PMC passes): time is not meaningful
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return 1.0
    for _ in range(2):
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
    return e0.elapsed_time(e1) / iters * 1e3     # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--only', default=None)
    ap.add_argument('--mm', action='store_true')
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--shape', action='append', default=[],
                    help='extra shape N,Cin,H,W,Cout,k,stride,levels (repeatable; replaces the table)')
    ap.add_argument('--variants', default='1,2,3,4,0', help='conv kernel families to time: 1-4 LDS-DMA configs, 0 register-staged; '
                    '+100*w: 256-column wgrad tiles of variant w (e.g. 209)')
    ap.add_argument('--ww', default=None, help='wide-wave fwd/dgrad variants to time per kernel family (ewvit_conv2d_set_ww), e.g. 0,1,2,3')
    ap.add_argument('--bnstats', action='store_true', help='time fwd against fwd with BN statistics in the epilogue')
    ap.add_argument('--w1', default=None, help='1x1 wgrad kernel settings to time (ewvit_conv2d_set_wgrad_1x1), '
                    'target_wg:min_ktiles:ring pairs, e.g. 0:4:3,256:4:3,128:4:3 (wgrad only)')
    ap.add_argument('--small', default=None, help='ewvit_conv2d_set_small_tiles settings to time, e.g. 0,1 (replaces --variants)')
    ap.add_argument('--eager', action='store_true', help='no HIP graph (for rocprofv3 --pmc passes)')
    ap.add_argument('--win', type=int, default=1, help='ewvit_conv2d_set_win: 1 windowed 3x3 kernels where they apply, 0 off')
    ap.add_argument('--cap', type=int, default=0, help='ewvit_set_grid_cap (the MWT stream runs under 128)')
    a = ap.parse_args()
    global EAGER
    EAGER = a.eager
    a.variants = [int(v) for v in a.variants.split(',')]
    small = None
    if a.small:
        small = [int(q) for q in a.small.split(',')]
        a.variants = [1 + 10000 * i for i in range(len(small))]
    w1 = None
    if a.w1:
        w1 = [tuple(int(q) for q in t.split(':')) for t in a.w1.split(',')]
        a.variants = [1 + 10000 * i for i in range(len(w1))]
    if a.ww is not None:      # variant v + 1000 * ww
        a.variants = [v + 1000 * int(w) for v in a.variants for w in a.ww.split(',')]
    import ewvit
    dev = torch.device('cuda', 0)
    from ewvit import _lib as L
    from ewvit.conv import _pack
    lib = L.load()
    lib.ewvit_conv2d_set_win(a.win)
    lib.ewvit_set_grid_cap(a.cap)
    shapes = SHAPES
    if a.shape:
        shapes = {f'shape{i}': tuple(int(v) for v in sh.split(',')) for i, sh in enumerate(a.shape)}
    for name, (N, Cin, H, W, Cout, k, s, lv) in shapes.items():
        if a.only and a.only not in name:
            continue
        Cx = Cin * lv
        z = torch.randn(N * lv, Cin, H, W, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = torch.randn(Cout, Cx, k, k, device=dev) / (k * k * Cx) ** 0.5
        gc, gs = (Cin, N * H * W * Cin) if lv > 1 else (0, 0)
        cp = Cx if lv > 1 else int(lib.ewvit_conv2d_fwd_pack_cin(N, H, W, Cx, Cout, k, s))
        wp, wpt = _pack(w, cp, True, True)
        Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
        y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        dy = torch.randn_like(y)
        dx = torch.empty_like(z)
        dw = torch.empty((Cout, Cx, k, k), device=dev)
        wsb = 0
        for wv in range(5):                    # largest workspace over the wgrad tile widths
            lib.ewvit_conv2d_set_wgrad_wide(wv)
            for t in (w1 or [(256, 4, 3)]):
                lib.ewvit_conv2d_set_wgrad_1x1(*t)
                wsb = max(wsb, lib.ewvit_conv2d_bwd_weight_workspace(N, H, W, Cx, Cout, k, s))
        lib.ewvit_conv2d_set_wgrad_1x1(256, 8, 2)
        lib.ewvit_conv2d_set_wgrad_wide(4)
        ws = torch.empty(wsb // 4, device=dev)

        flops = 2.0 * N * Ho * Wo * Cout * k * k * Cx

        def fwd():
            L.call('ewvit_conv2d_fwd', L.ptr(z), L.ptr(wp), None, L.ptr(y), N, H, W, Cx, Cout, k, s, gc, gs,
                   L.stream(y))

        def dgrad():
            L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx), N, H, W, Cx, Cout, k, s, gc, gs,
                   L.stream(y))

        rows_bn = int(lib.ewvit_conv2d_fwd_bn_rows(N, H, W, Cx, Cout, k, s))
        part = torch.empty(max(1, (N * Ho * Wo + max(rows_bn, 1) - 1) // max(rows_bn, 1)), 2 * Cout, device=dev)
        shift = torch.zeros(Cout, device=dev)
        shift_out = torch.empty(Cout, device=dev)

        def fwd_bn():
            L.call('ewvit_conv2d_fwd_bn', L.ptr(z), L.ptr(wp), None, L.ptr(y), N, H, W, Cx, Cout, k, s, gc, gs,
                   L.ptr(shift), L.ptr(part), L.ptr(shift_out), L.stream(y))

        def wgrad():
            L.call('ewvit_conv2d_bwd_weight', L.ptr(z), L.ptr(dy), L.ptr(dw), None, 0, N, H, W, Cx, Cout, k, s,
                   gc, gs, Cx, dw.stride(0), dw.stride(1), dw.stride(3), L.ptr(ws), L.stream(y))
        rows = {}
        for r in range(a.rounds):              # interleaved A/B rounds in one process
            for v in a.variants:
                if small is not None:
                    lib.ewvit_conv2d_set_small_tiles(small[v // 10000])
                    lib.ewvit_conv2d_set_glds(1)
                    for pn, fn in (('fwd', fwd), ('dgrad', dgrad)):
                        rows.setdefault((v, pn), []).append(graph_time(fn, a.iters))
                    continue
                if w1:
                    lib.ewvit_conv2d_set_wgrad_1x1(*w1[v // 10000])
                    lib.ewvit_conv2d_set_glds(1)
                    rows.setdefault((v, 'wgrad'), []).append(graph_time(wgrad, a.iters))
                    continue
                lib.ewvit_conv2d_set_glds(v % 100)
                lib.ewvit_conv2d_set_wgrad_wide(v % 1000 // 100)     # 0 = 128-column tiles, 4 = auto
                if a.ww is not None:
                    lib.ewvit_conv2d_set_ww(v // 1000)
                phases = (('fwd', fwd), ('dgrad', dgrad), ('wgrad', wgrad))
                if a.bnstats and rows_bn > 0:
                    phases = (('fwd', fwd), ('fwd_bn', fwd_bn))
                for pn, fn in phases:
                    rows.setdefault((v, pn), []).append(graph_time(fn, a.iters))
        lib.ewvit_conv2d_set_glds(1)
        lib.ewvit_conv2d_set_wgrad_wide(4)
        if a.ww is not None:
            lib.ewvit_conv2d_set_ww(0)
        lib.ewvit_conv2d_set_wgrad_1x1(256, 8, 2)
        lib.ewvit_conv2d_set_small_tiles(1)
        for v in a.variants:
            parts = []
            if small is not None:
                print(f'{name:15s} [small {small[v // 10000]}] fwd {min(rows[(v, "fwd")]):8.1f} us | dgrad '
                      f'{min(rows[(v, "dgrad")]):8.1f} us', flush=True)
                continue
            if w1:
                t = min(rows[(v, 'wgrad')])
                print(f'{name:15s} [w1 {":".join(map(str, w1[v // 10000])):>10s}] wgrad {t:8.1f} us {flops / t / 1e6:6.0f} TF/s',
                      flush=True)
                continue
            for pn in (('fwd', 'fwd_bn') if a.bnstats and rows_bn > 0 else ('fwd', 'dgrad', 'wgrad')):
                t = min(rows[(v, pn)])
                parts.append(f'{pn} {t:8.1f} us {flops / t / 1e6:6.0f} TF/s')
            print(f'{name:15s} [{f"glds{v}" if v else "regs "}] ' + ' | '.join(parts), flush=True)
        if a.mm and k == 1 and s == 1:
            M = N * H * W
            x2 = torch.randn(M, Cin, device=dev, dtype=torch.bfloat16)
            w2 = torch.randn(Cout, Cin, device=dev, dtype=torch.bfloat16)
            d2 = torch.randn(M, Cout, device=dev, dtype=torch.bfloat16)
            t1 = graph_time(lambda: torch.mm(x2, w2.t()), a.iters)
            t2 = graph_time(lambda: torch.mm(d2, w2), a.iters)
            t3 = graph_time(lambda: torch.mm(d2.t(), x2), a.iters)
            dwo = torch.empty(Cout, Cin, device=dev)
            try:
                t4 = graph_time(lambda: torch.mm(d2.t(), x2, out_dtype=torch.float32, out=dwo), a.iters)
            except Exception as e:          # out_dtype not supported on this build
                print(f'{name:15s} [hipBLASLt] fp32-out wgrad: {type(e).__name__}: {e}', flush=True)
                t4 = float('nan')
            print(f'{name:15s} [hipBLASLt] fwd {t1:8.1f} us | dgrad {t2:8.1f} us | wgrad {t3:8.1f} us | '
                  f'wgrad fp32 out {t4:8.1f} us', flush=True)


if __name__ == '__main__':
    main()
