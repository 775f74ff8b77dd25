"""The windowed 3x3 weight gradient's tap-split 8-wave variant (csrc/convwin.hip
conv_wgrad_win_kernel<.., TS = true>, ewvit_conv2d_set_wgrad_tap_split): waves 0-3 own taps 0-4,
waves 4-7 taps 5-8 of the same (co half, ci half) blocks, so every dW entry is the same MFMA chain
over the same pixel tiles as the 4-wave kernel — dW and the bias gradient must be BIT-IDENTICAL
to it, with and without the input transform (XF), under a grid cap (persistent walk), and against
torch float64 of the same bf16 operands (the MWT conv shapes of reference network/mwt.py:60-72).
Setting 2 (12 waves, one kernel row per wave group, strided DMA pieces) is held to the same bar."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('N,C,H,W,Cout,levels,xf,bias,cap', [
    (2, 128, 32, 48, 128, 3, True, True, 0),     # multiscale fusion class: 3 levels, transform + bias
    (2, 128, 32, 32, 128, 1, False, True, 0),    # plain, bias
    (1, 64, 48, 32, 256, 1, False, False, 0),    # two co tiles, no bias
    (2, 128, 32, 32, 128, 2, True, False, 5),    # transform, persistent walk under a grid cap
    (1, 192, 32, 64, 128, 1, False, True, 7),    # 6 ci blocks, ragged split boundaries
])
def test_tap_split_bit_identical(N, C, H, W, Cout, levels, xf, bias, cap):
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    lib = L.load()
    g = torch.Generator().manual_seed(C + H + 3 * levels + cap)
    NL, Cx = N * levels, C * levels
    z = torch.randn(NL, C, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    coef = torch.stack([torch.rand(levels, C, generator=g) + 0.5, torch.randn(levels, C, generator=g) * 0.5], 1)
    coef = coef.to(DEV).contiguous()
    dy = torch.randn(N, Cout, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gc, gs = (C, N * H * W * C) if levels > 1 or xf else (Cx, 0)
    assert lib.ewvit_conv2d_xf_ok(N, H, W, Cx, Cout, 3, 1, gc, gs) == 1    # the windowed wgrad takes it
    prev_cap = lib.ewvit_set_grid_cap(cap)
    out = {}
    try:
        for ts in (0, 1, 2):
            prev = lib.ewvit_conv2d_set_wgrad_tap_split(ts)
            try:
                dw = torch.full((Cout, Cx, 3, 3), float('nan'), device=DEV)
                db = torch.full((Cout,), float('nan'), device=DEV) if bias else None
                ws = torch.empty(int(lib.ewvit_conv2d_bwd_weight_workspace(N, H, W, Cx, Cout, 3, 1)) // 4, device=DEV)
                if xf:
                    L.call('ewvit_conv2d_bwd_weight_xf', L.ptr(z), L.ptr(dy), L.ptr(dw), L.ptr(db) if bias else None, 0,
                           N, H, W, Cx, Cout, gc, gs, L.ptr(coef), Cx, dw.stride(0), dw.stride(1), dw.stride(3),
                           L.ptr(ws), L.stream(dw))
                else:
                    L.call('ewvit_conv2d_bwd_weight', L.ptr(z), L.ptr(dy), L.ptr(dw), L.ptr(db) if bias else None, 0,
                           N, H, W, Cx, Cout, 3, 1, gc, gs, Cx, dw.stride(0), dw.stride(1), dw.stride(3), L.ptr(ws),
                           L.stream(dw))
                torch.cuda.synchronize()
                out[ts] = (dw, db)
            finally:
                lib.ewvit_conv2d_set_wgrad_tap_split(prev)
    finally:
        lib.ewvit_set_grid_cap(prev_cap)
    for ts in (1, 2):
        assert torch.equal(out[0][0], out[ts][0]), ('dW', ts)
        if bias:
            assert torch.equal(out[0][1], out[ts][1]), ('db', ts)
    # torch (float64) of the same operands (the transform applied in float64, bf16-rounded as the kernel's staging)
    zl = z.double().view(levels, N, C, H, W)
    if xf:
        cd = coef.double()
        zl = torch.relu(zl * cd[:, 0].view(levels, 1, C, 1, 1) + cd[:, 1].view(levels, 1, C, 1, 1))
    a = zl.float().to(torch.bfloat16).double().permute(1, 0, 2, 3, 4).reshape(N, Cx, H, W)
    a.requires_grad_(True)
    w = torch.zeros(Cout, Cx, 3, 3, device=DEV, dtype=torch.float64, requires_grad=True)
    torch.nn.functional.conv2d(a, w, padding=1).backward(dy.double())
    ref = w.grad.float()
    err = (out[1][0] - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item() + 1e-4, err
    if bias:
        torch.testing.assert_close(out[1][1], dy.float().sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
