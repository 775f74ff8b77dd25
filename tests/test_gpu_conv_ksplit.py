"""Split K of the LDS-DMA 1x1 forward / input gradient (csrc/conv.hip launch_glds, FwdArgs::ksplit,
conv_splitk_epi_kernel) on the backbone's long-K 1x1 shapes (EfficientNetV2-S MBConv project
forward / expand input gradient of stages 4-6 and the head conv, sfe.py:111-113) plus a ragged
row count, through the C-ABI:
  * split (ewvit_conv2d_set_ksplit(1); off by default) and unsplit outputs against torch fp32 of the
    same bf16 operands (bf16 rounding: 2^-8 of the largest output), and against each other
    (one bf16 ulp: the fp32 sums differ only in order);
  * the forward's BatchNorm statistics partial rows and the input gradient's backward sums
    (the BatchNorm + SiLU before the conv) against fp64 sums of the stored bf16 output."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _L():
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    L.load()
    return L


def bf(t):
    return t.to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)


# on, up to 8 splits of >= 4 K-tiles (16 * min K-tiles + max splits): S = 4 / 3 / 2 / 5 / 4 on
# the shapes below; KS_DEFAULT restores the library's limits (<= 2 splits of >= 8 K-tiles)
KS_ON, KS_DEFAULT = 16 * 4 + 8, 16 * 8 + 2
SHAPES = [(64, 7, 7, 1536, 256), (64, 14, 14, 960, 160), (64, 14, 14, 512, 128), (64, 7, 7, 1280, 256),
          (3, 7, 7, 1536, 256)]


def _ulp_close(a, b, ref):
    scale = float(ref.abs().max())
    assert float((a.float() - ref).abs().max()) <= 2 ** -8 * scale * 2
    assert float((b.float() - ref).abs().max()) <= 2 ** -8 * scale * 2
    # the two roundings of fp32 sums that differ only in order: at most one bf16 ulp apart
    # (plus an absolute floor for outputs that cancel to ~0, where the order of the fp32 sums
    # shows: ~sqrt(K) fp32 ulps of the terms)
    d = (a.float() - b.float()).abs()
    ulp = torch.maximum(a.float().abs(), b.float().abs()) * 2 ** -7 + 1e-5 * scale
    assert bool((d <= ulp).all()), float((d - ulp).max())


@pytest.mark.parametrize('N,H,W,K,Nout', SHAPES)
def test_ksplit_forward_with_statistics(N, H, W, K, Nout):
    """conv2d_fwd_bn: y = x W^T (+ bias), per m-tile sum (y - K) and sum (y - K)^2."""
    L = _L()
    lib = L.load()
    g = torch.Generator().manual_seed(K + Nout + N)
    x = bf(torch.randn(N, K, H, W, generator=g))
    w = (torch.randn(Nout, K, generator=g) / K ** 0.5).to(DEV, torch.bfloat16).contiguous()
    bias = (torch.randn(Nout, generator=g) * 0.1).to(DEV)
    shift = (torch.randn(Nout, generator=g) * 0.05).to(DEV)
    rows = int(lib.ewvit_conv2d_fwd_bn_rows(N, H, W, K, Nout, 1, 1))
    assert rows > 0
    nrc = (N * H * W + rows - 1) // rows
    outs = []
    for split in (KS_ON, 0):
        prev = lib.ewvit_conv2d_set_ksplit(split)
        try:
            y = torch.empty(N, Nout, H, W, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
            part = torch.full((nrc, 2 * Nout), float('nan'), device=DEV)
            so = torch.empty(Nout, device=DEV)
            L.call('ewvit_conv2d_fwd_bn', L.ptr(x), L.ptr(w), L.ptr(bias), L.ptr(y), N, H, W, K, Nout, 1, 1, K, 0,
                   L.ptr(shift), L.ptr(part), L.ptr(so), L.stream(y))
            torch.cuda.synchronize()
        finally:
            lib.ewvit_conv2d_set_ksplit(KS_DEFAULT)        # the default limits back
            lib.ewvit_conv2d_set_ksplit(prev)
        outs.append((y, part, so))
    xm = x.permute(0, 2, 3, 1).reshape(-1, K).double()
    ref = (xm @ w.double().t() + bias.double()).float()
    ya, yb = (o[0].permute(0, 2, 3, 1).reshape(-1, Nout) for o in outs)
    _ulp_close(ya, yb, ref)
    for y2, part, so in outs:
        yd = y2.permute(0, 2, 3, 1).reshape(-1, Nout).double() - shift.double()
        s1, s2 = yd.sum(0), (yd * yd).sum(0)
        assert not torch.isnan(part).any()
        assert float((part[:, :Nout].double().sum(0) - s1).abs().max()) <= 1e-5 * float(yd.abs().sum(0).max())
        assert float((part[:, Nout:].double().sum(0) - s2).abs().max()) <= 1e-5 * float(s2.abs().max())
        assert torch.equal(so, shift)


@pytest.mark.parametrize('N,H,W,K,Nin', SHAPES)
def test_ksplit_input_gradient_with_bn_sums(N, H, W, K, Nin):
    """conv2d_bwd_data_bn (K = the conv's output channels): dx = dy W, and the backward sums
    of the BatchNorm + SiLU that produced the conv's input, per m-tile."""
    L = _L()
    lib = L.load()
    g = torch.Generator().manual_seed(K * 3 + Nin + N)
    dy = bf(torch.randn(N, K, H, W, generator=g))
    wt = torch.randn(K, Nin, generator=g) / K ** 0.5                # forward weight [Cout = K][Cin = Nin]
    wpt = wt.t().contiguous().to(DEV, torch.bfloat16)              # [Cin][1][Cout]
    bx = bf(torch.randn(N, Nin, H, W, generator=g) * 1.2 - 0.1)
    gamma = (torch.randn(Nin, generator=g) * 0.3 + 1).to(DEV)
    beta = (torch.randn(Nin, generator=g) * 0.2).to(DEV)
    xb = bx.float()
    mean = xb.mean((0, 2, 3)).contiguous()
    invstd = torch.rsqrt(xb.var((0, 2, 3), unbiased=False) + 1e-3).contiguous()
    rows = int(lib.ewvit_conv2d_bwd_bn_rows(N, H, W, Nin, K, 1, 1))
    outs = []
    for split in (KS_ON, 0):
        prev = lib.ewvit_conv2d_set_ksplit(split)
        try:
            dx = torch.empty_like(bx)
            dx2 = torch.empty_like(bx)
            part = torch.full((rows, 2 * Nin), float('nan'), device=DEV)
            nrc = ctypes.c_int(0)
            L.call('ewvit_conv2d_bwd_data_bn', L.ptr(dy), L.ptr(wpt), L.ptr(dx), None, N, H, W, Nin, K, 1, 1, 0, 0,
                   L.ptr(bx), L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), 2, None, 0, L.ptr(part),
                   ctypes.byref(nrc), L.stream(dy))
            L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx2), N, H, W, Nin, K, 1, 1, 0, 0,
                   L.stream(dy))
            torch.cuda.synchronize()
        finally:
            lib.ewvit_conv2d_set_ksplit(KS_DEFAULT)        # the default limits back
            lib.ewvit_conv2d_set_ksplit(prev)
        assert torch.equal(dx, dx2)
        outs.append((dx, part[:nrc.value]))
    dym = dy.permute(0, 2, 3, 1).reshape(-1, K).double()
    ref = (dym @ wt.double().to(DEV)).float()
    da, db = (o[0].permute(0, 2, 3, 1).reshape(-1, Nin) for o in outs)
    _ulp_close(da, db, ref)
    for dx, part in outs:
        d = dx.double().cpu()
        xh = (bx.double().cpu() - mean.double().cpu().view(1, -1, 1, 1)) * invstd.double().cpu().view(1, -1, 1, 1)
        z = xh * gamma.double().cpu().view(1, -1, 1, 1) + beta.double().cpu().view(1, -1, 1, 1)
        s = torch.sigmoid(z)
        gr = d * s * (1 + z * (1 - s))
        ra, rb = gr.sum((0, 2, 3)), (gr * xh).sum((0, 2, 3))
        ma, mb = gr.abs().sum((0, 2, 3)), (gr * xh).abs().sum((0, 2, 3))
        pa, pb = part[:, :Nin].double().sum(0).cpu(), part[:, Nin:].double().sum(0).cpu()
        assert float(((pa - ra).abs() / ma.clamp_min(1e-12)).max()) < 1e-5
        assert float(((pb - rb).abs() / mb.clamp_min(1e-12)).max()) < 1e-5


def test_ksplit_switch_restores():
    """off by default (measured slower in the step, conv.hip g_ksplit)"""
    L = _L()
    lib = L.load()
    assert lib.ewvit_conv2d_set_ksplit(1) == 0
    assert lib.ewvit_conv2d_set_ksplit(0) == 1
