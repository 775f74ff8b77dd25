"""The windowed 3x3 stride-1 conv kernels (csrc/convwin.hip) through the C-ABI.

They walk K in the generic LDS-DMA kernel's order (64-channel block outer, tap inner) with
the same MFMA operand order, so outputs and input gradients must be BIT-IDENTICAL to
ewvit_conv2d_set_win(0) runs (which are themselves checked against torch fp32 in
test_gpu_conv.py); the forward's BatchNorm partial sums (one partial row per 16 x 16 block)
equal the generic kernel's (per 128 rows) to fp32 summation order (1e-6 relative).  Cases:
plain and level-grouped inputs (mwt.py:112's channel concatenation read in place), several
column tiles (the 384-channel input gradient), 1-4 channel blocks, persistent walks under a
grid cap, and a map whose blocks cover the image borders on every side.

The one exception is the 64-column input gradient (hf_conv['fusion'], 128 -> 64): its k-split
form sums each K-tile's two k32 halves in different waves and adds them at the tile's end, so
it is checked against the fp32 conv input gradient (2^-7 of scale, bf16 output) and against the
generic kernel to one bf16 ulp instead."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _run(lib, L, win, cap, z, wp, wpt, bias, dy, shift, N, H, W, Cx, Cout, gc, gs, stats):
    lib.ewvit_conv2d_set_win(win)
    prev = lib.ewvit_set_grid_cap(cap)
    try:
        y = torch.empty((N, Cout, H, W), dtype=torch.bfloat16, device=DEV, memory_format=torch.channels_last)
        dx = torch.empty_like(z)
        L.call('ewvit_conv2d_fwd', L.ptr(z), L.ptr(wp), L.ptr(bias), L.ptr(y), N, H, W, Cx, Cout, 3, 1, gc, gs,
               L.stream(y))
        L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx), N, H, W, Cx, Cout, 3, 1, gc, gs,
               L.stream(y))
        sums = None
        if stats:
            rows = int(lib.ewvit_conv2d_fwd_bn_rows(N, H, W, Cx, Cout, 3, 1))
            assert rows == 256 if win else rows in (64, 128)      # the generic kernel: 64-row tiles on small grids
            M = N * H * W
            part = torch.zeros((M + rows - 1) // rows, 2 * Cout, device=DEV)
            so = torch.empty(Cout, device=DEV)
            y2 = torch.empty_like(y)
            L.call('ewvit_conv2d_fwd_bn', L.ptr(z), L.ptr(wp), L.ptr(bias), L.ptr(y2), N, H, W, Cx, Cout, 3, 1,
                   gc, gs, L.ptr(shift), L.ptr(part), L.ptr(so), L.stream(y))
            torch.cuda.synchronize()
            assert torch.equal(y2, y)
            assert torch.equal(so, shift)
            sums = part.double().sum(0)
        torch.cuda.synchronize()
        return y, dx, sums
    finally:
        lib.ewvit_set_grid_cap(prev)
        lib.ewvit_conv2d_set_win(1)


@pytest.mark.parametrize('N,Cin,H,W,Cout,levels,cap', [
    (2, 64, 32, 48, 128, 1, 0),       # the hf fusion conv's shape class, 6 x 16^2 blocks per image
    (1, 128, 16, 32, 128, 3, 0),      # multiscale_fusion: level-major input, 6 channel blocks
    (4, 64, 32, 32, 128, 2, 5),       # 2 levels, persistent walk (cap 5 -> 8 workgroups, 16 tiles)
    (1, 128, 48, 16, 64, 1, 0),       # 64-channel output: forward on the generic kernel, dgrad windowed
    (2, 256, 32, 32, 128, 1, 16),     # 4 channel blocks, capped
    (1, 128, 16, 16, 256, 3, 0),      # 2 column tiles with bias + statistics (config 4), dgrad 3 x 128 cols
    (4, 64, 32, 32, 128, 1, 5),       # k-split dgrad, persistent walk over both window buffers
    (3, 64, 48, 16, 128, 1, 0),       # k-split dgrad, 3 blocks per image column
])
def test_window_bit_identical(N, Cin, H, W, Cout, levels, cap):
    import ewvit
    from ewvit import _lib as L
    from ewvit.conv import _pack
    lib = L.load()
    g = torch.Generator().manual_seed(N * 131 + Cin + H)
    Cx = Cin * levels
    z = torch.randn(N * levels, Cin, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cx, 3, 3, generator=g) / (9 * Cx) ** 0.5).to(DEV)
    bias = torch.randn(Cout, generator=g).to(DEV)
    dy = torch.randn(N, Cout, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    shift = (torch.randn(Cout, generator=g) * 0.1).to(DEV)
    gc, gs = (Cin, N * H * W * Cin) if levels > 1 else (0, 0)
    wp, wpt = _pack(w, Cx, True, True)
    stats = Cout in (128, 256)
    y0, d0, s0 = _run(lib, L, 0, cap, z, wp, wpt, bias, dy, shift, N, H, W, Cx, Cout, gc, gs, stats)
    y1, d1, s1 = _run(lib, L, 1, cap, z, wp, wpt, bias, dy, shift, N, H, W, Cx, Cout, gc, gs, stats)
    assert torch.equal(y0, y1), float((y0.float() - y1.float()).abs().max())
    if Cx == 64:
        # k-split: the fp32 input gradient, and the generic kernel to one bf16 ulp
        dref = torch.nn.grad.conv2d_input(z.shape, w.to(torch.bfloat16).float(), dy.float(), padding=1)
        derr = float((d1.float() - dref).abs().max() / dref.abs().max())
        assert derr < 2 ** -7, derr
        # (plus fp32 summation-order noise where the sum cancels to near zero)
        ulp = torch.maximum(d0.float().abs(), d1.float().abs()) * 2 ** -7 + 2 ** -16 * float(dref.abs().max())
        assert bool(((d0.float() - d1.float()).abs() <= ulp).all())
        assert float((d0.float() - d1.float()).abs().mean()) < 1e-3 * float(dref.abs().mean())
    else:
        assert torch.equal(d0, d1), float((d0.float() - d1.float()).abs().max())
    if stats:
        assert float((s0 - s1).abs().max() / s0.abs().max()) < 1e-6
    # and the generic result is the conv itself (bf16 operands, fp32 accumulation)
    ref = torch.nn.functional.conv2d(torch.cat(z.float().chunk(levels), 1) if levels > 1 else z.float(), w.to(
        torch.bfloat16).float(), bias, padding=1)
    err = float((y1.float() - ref).abs().max() / ref.abs().max())
    assert err < 2 ** -7, err
