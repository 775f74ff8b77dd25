"""The windowed 3x3 stride-1 conv kernels (csrc/convwin.hip) against the generic LDS-DMA
kernels (ewvit_conv2d_set_win 0 / 1) on the MWT shapes: outputs and input gradients must be
bit-identical (same K order, same MFMA operand order); the forward's BatchNorm partial sums
(one row per 16 x 16 block instead of per 128 rows) agree to fp32 summation order.  Then
both are timed as ITERS launches replayed from one HIP graph (interleaved rounds).
Usage: python tools/win_bench.py [--iters N] [--rounds R] [--only NAME] [--check-only]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))

# name: (N, Cin per level, H, W, Cout, levels)
SHAPES = {
    'small_plain': (2, 64, 32, 48, 128, 1),
    'small_grouped': (2, 128, 16, 32, 128, 3),
    'small_dgrad': (1, 128, 48, 16, 64, 1),
    'mwt_multiscale': (64, 128, 112, 112, 128, 3),
    'mwt_fusion': (192, 64, 112, 112, 128, 1),
    'c4_multiscale': (32, 256, 192, 192, 256, 3),
    'c4_fusion': (96, 64, 192, 192, 256, 1),
}


VARIANTS = (0, 1)      # ewvit_conv2d_set_win: generic LDS-DMA, windowed


def graph_time(fn, iters):
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
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--only', default=None)
    ap.add_argument('--check-only', action='store_true')
    ap.add_argument('--cap', type=int, default=0, help='grid cap for the timed launches')
    ap.add_argument('--profile', default=None, help='fwd|fwd_bn|dgrad|wgrad: only run that phase 5x eagerly per '
                    'variant in --variants (rocprofv3 passes)')
    ap.add_argument('--variants', default=None, help='comma list of ewvit_conv2d_set_win variants for --profile')
    a = ap.parse_args()
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    from ewvit.conv import _pack
    lib = L.load()
    dev = torch.device('cuda', 0)
    bad = 0
    for name, (N, Cin, H, W, Cout, lv) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        torch.manual_seed(hash(name) % 1000)
        Cx = Cin * lv
        k = 3
        z = torch.randn(N * lv, Cin, H, W, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = torch.randn(Cout, Cx, k, k, device=dev) / (k * k * Cx) ** 0.5
        bias = torch.randn(Cout, device=dev)
        gc, gs = (Cin, N * H * W * Cin) if lv > 1 else (0, 0)
        wp, wpt = _pack(w, Cx, True, True)
        y = torch.empty((N, Cout, H, W), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        dy = torch.randn_like(y)
        dx = torch.empty_like(z)
        shift = torch.randn(Cout, device=dev) * 0.1
        shift_out = torch.empty(Cout, device=dev)
        M = N * H * W
        part = torch.empty((M + 127) // 128, 2 * Cout, device=dev)
        flops = 2.0 * M * Cout * k * k * Cx
        use_bias = Cout <= 512

        def fwd():
            L.call('ewvit_conv2d_fwd', L.ptr(z), L.ptr(wp), L.ptr(bias) if use_bias else None, L.ptr(y), N, H, W,
                   Cx, Cout, k, 1, gc, gs, L.stream(y))

        def fwd_bn():
            L.call('ewvit_conv2d_fwd_bn', L.ptr(z), L.ptr(wp), L.ptr(bias) if use_bias else None, L.ptr(y), N, H,
                   W, Cx, Cout, k, 1, gc, gs, L.ptr(shift), L.ptr(part), L.ptr(shift_out), L.stream(y))

        def dgrad():
            L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx), N, H, W, Cx, Cout, k, 1, gc, gs,
                   L.stream(y))

        dw = torch.empty((Cout, Cx, k, k), device=dev)
        db = torch.empty(Cout, device=dev)
        wsb = 0
        for v in (0, 1):
            lib.ewvit_conv2d_set_win(v)
            wsb = max(wsb, lib.ewvit_conv2d_bwd_weight_workspace(N, H, W, Cx, Cout, k, 1))
        lib.ewvit_conv2d_set_win(1)
        wsp = torch.empty(wsb // 4 + 1, device=dev)

        def wgrad():
            L.call('ewvit_conv2d_bwd_weight', L.ptr(z), L.ptr(dy), L.ptr(dw), L.ptr(db), 0, N, H, W, Cx, Cout, k, 1,
                   gc, gs, Cx, dw.stride(0), dw.stride(1), dw.stride(3), L.ptr(wsp), L.stream(y))

        if a.profile:
            fn = dict(fwd=fwd, fwd_bn=fwd_bn, dgrad=dgrad, wgrad=wgrad)[a.profile]
            for v in ([int(x) for x in a.variants.split(',')] if a.variants else [1]):
                lib.ewvit_conv2d_set_win(v)
                for _ in range(5):
                    fn()
                torch.cuda.synchronize()
            lib.ewvit_conv2d_set_win(1)
            print(f'{name}: profiled {a.profile}', flush=True)
            continue
        res = {}
        wres = {}
        for v in (0, 1):
            lib.ewvit_conv2d_set_win(v)
            wgrad()
            torch.cuda.synchronize()
            wres[v] = (dw.clone(), db.clone())
            lib.ewvit_conv2d_set_win(v)
            fwd()
            yf = y.clone()
            dgrad()
            dxv = dx.clone()
            rows = int(lib.ewvit_conv2d_fwd_bn_rows(N, H, W, Cx, Cout, k, 1))
            sums = None
            if use_bias and rows > 0:
                part.zero_()
                fwd_bn()
                nr = (M + rows - 1) // rows
                sums = part[:nr].double().sum(0)
            torch.cuda.synchronize()
            res[v] = (yf, dxv, sums, rows)
        lib.ewvit_conv2d_set_win(1)
        y0, d0, s0, r0 = res[0]
        y1, d1, s1, r1 = res[1]
        ok_y = torch.equal(y0, y1)
        ok_d = torch.equal(d0, d1)
        msg = f'{name:15s} fwd {"bit-equal" if ok_y else "DIFF %.3g" % (y0.float() - y1.float()).abs().max().item()}'
        msg += f' | dgrad {"bit-equal" if ok_d else "DIFF %.3g" % (d0.float() - d1.float()).abs().max().item()}'
        if s0 is not None and s1 is not None:
            e = float((s0 - s1).abs().max() / s0.abs().max())
            msg += f' | bn sums rel {e:.2e} (rows {r0} -> {r1})'
            if e > 1e-5:
                bad += 1
        if not (ok_y and ok_d):
            bad += 1
        ew = float((wres[0][0] - wres[1][0]).abs().max() / wres[0][0].abs().max())
        eb = float((wres[0][1] - wres[1][1]).abs().max() / wres[0][1].abs().max())
        msg += f' | wgrad rel {ew:.2e} bias rel {eb:.2e}'
        if ew > 1e-5 or eb > 1e-5:
            bad += 1
        print(msg, flush=True)
        if a.check_only or name.startswith('small'):
            continue
        t = {}
        prev_cap = lib.ewvit_set_grid_cap(a.cap)
        for r in range(a.rounds):
            for v in VARIANTS:
                lib.ewvit_conv2d_set_win(v)
                for pn, fn in (('fwd', fwd), ('fwd_bn', fwd_bn), ('dgrad', dgrad), ('wgrad', wgrad)):
                    if pn == 'fwd_bn' and not use_bias:
                        continue
                    t.setdefault((v, pn), []).append(graph_time(fn, a.iters))
        lib.ewvit_set_grid_cap(prev_cap)
        lib.ewvit_conv2d_set_win(1)
        for v in VARIANTS:
            parts = [f'{pn} {min(ts):8.1f} us {flops / min(ts) / 1e6:6.0f} TF/s'
                     for (vv, pn), ts in t.items() if vv == v]
            print(f'{name:15s} [{("glds", "win ")[v]}] ' + ' | '.join(parts), flush=True)
    print('FAILURES', bad if bad else 'none', flush=True)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()
