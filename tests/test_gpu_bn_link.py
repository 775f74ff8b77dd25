"""BatchNorm statistics summed by the neighbouring kernels (csrc/depthwise.hip
dw_row_bn_kernel, csrc/conv.hip dgrad epilogue, csrc/batchnorm.hip ewvit_bn_bwd_partials):
the MBConv block's BatchNorms with no statistics / reduction pass of their own.

Kernel level (through the C-ABI): the stored outputs are bit-identical to the plain kernels
(the sums are an epilogue on the same values), and the partial rows add up to the fp64 sums
of those stored values (1e-5 of the sum of magnitudes: fp32 adds in a fixed order).
ewvit_bn_bwd_partials vs ewvit_bn_bwd: dx within 2 bf16 ulps (the two reductions add the same
terms in different orders, so the finalised means differ in the last fp32 bits).
Module level: four MBConv blocks with the links on vs off (the A/B switches) — outputs,
running statistics and every gradient equal to the tolerance of those orders (outputs cosine
>= 0.99999 and max 2e-2 of scale, gradients cosine >= 0.999); all 30 MBConv blocks of stages
4-6: the fused launches are the ones that ran, one per BatchNorm the links can serve.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _L():
    import ewvit
    return ewvit._lib


def bf(t):
    return t.to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)


def sums_close(part, ref_a, ref_b, mag_a, mag_b):
    """part [rows][2C] summed over rows vs fp64 references (per channel)."""
    p = part.double().sum(0).cpu()
    C = ref_a.numel()
    ea = float(((p[:C] - ref_a).abs() / (mag_a + 1e-30)).max())
    eb = float(((p[C:] - ref_b).abs() / (mag_b + 1e-30)).max())
    return ea, eb


DW_SHAPES = [(16, 1536, 7, 7, 1), (16, 960, 14, 14, 1), (8, 256, 28, 28, 2), (4, 200, 9, 11, 1), (3, 64, 5, 5, 2)]


@pytest.mark.parametrize('N,C,H,W,stride', DW_SHAPES)
def test_dw_fwd_bn(N, C, H, W, stride):
    L = _L()
    g = torch.Generator().manual_seed(C + H)
    x = bf(torch.randn(N, C, H, W, generator=g))
    w = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).to(DEV).contiguous()
    shift = (torch.randn(C, generator=g) * 0.2).to(DEV)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y0 = torch.empty(N, C, Ho, Wo, dtype=torch.bfloat16, device=DEV, memory_format=torch.channels_last)
    y1 = torch.empty_like(y0)
    L.call('ewvit_dwconv3x3_fwd', L.ptr(x), L.ptr(w), L.ptr(y0), N, H, W, C, stride, 1, L.BF16, L.stream(x))
    nrc = int(L.load().ewvit_dwconv3x3_bn_rows(N, H, W, C, stride, 0))
    assert nrc == (N * Ho + 31) // 32          # row kernel (the per-pixel form is off by default)
    part = torch.full((nrc, 2 * C), float('nan'), device=DEV)
    so = torch.full((C,), float('nan'), device=DEV)
    L.call('ewvit_dwconv3x3_fwd_bn', L.ptr(x), L.ptr(w), L.ptr(y1), N, H, W, C, stride, L.ptr(shift), L.ptr(part),
           L.ptr(so), L.stream(x))
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(so, shift)
    d = (y1.double().cpu() - shift.double().cpu().view(1, C, 1, 1))
    ra, rb = d.sum((0, 2, 3)), (d * d).sum((0, 2, 3))
    ea, eb = sums_close(part, ra, rb, d.abs().sum((0, 2, 3)), rb)
    assert ea < 1e-5 and eb < 1e-5, (ea, eb)


def _bwd_ref(dx, bx, mean, invstd, gamma, beta, act, rscale=None, hw=1):
    """fp64 g and g*xhat sums per channel of the stored dx (bf16) — bn_bwd_reduce_kernel's terms."""
    d, x = dx.double().cpu(), bx.double().cpu()
    C = d.shape[1]
    xh = (x - mean.double().cpu().view(1, C, 1, 1)) * invstd.double().cpu().view(1, C, 1, 1)
    if act == 2:
        z = xh * gamma.double().cpu().view(1, C, 1, 1) + beta.double().cpu().view(1, C, 1, 1)
        s = torch.sigmoid(z)
        gr = d * s * (1 + z * (1 - s))
    elif act == 1:
        z = xh * gamma.double().cpu().view(1, C, 1, 1) + beta.double().cpu().view(1, C, 1, 1)
        gr = d * (z > 0).double()
    else:
        gr = d
    if rscale is not None:
        gr = gr * rscale.double().cpu().view(-1, 1, 1, 1)
    return gr.sum((0, 2, 3)), (gr * xh).sum((0, 2, 3)), gr.abs().sum((0, 2, 3)), (gr * xh).abs().sum((0, 2, 3))


def _bn_stats(bx):
    x = bx.float()
    mean = x.mean((0, 2, 3))
    invstd = torch.rsqrt(x.var((0, 2, 3), unbiased=False) + 1e-3)
    return mean.contiguous(), invstd.contiguous()


@pytest.mark.parametrize('N,C,H,W', [(16, 1536, 7, 7), (16, 960, 14, 14), (4, 200, 9, 11), (2, 64, 30, 30)])
def test_dw_bwd_data_bn(N, C, H, W):
    L = _L()
    g = torch.Generator().manual_seed(C * 3 + H)
    dy = bf(torch.randn(N, C, H, W, generator=g))
    bx = bf(torch.randn(N, C, H, W, generator=g) * 1.5 + 0.3)
    w = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).to(DEV).contiguous()
    gamma = (torch.randn(C, generator=g) * 0.3 + 1).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV)
    mean, invstd = _bn_stats(bx)
    dx0 = torch.empty_like(dy)
    dx1 = torch.empty_like(dy)
    L.call('ewvit_dwconv3x3_bwd_data', L.ptr(dy), L.ptr(w), L.ptr(dx0), N, H, W, C, 1, 1, L.BF16, L.stream(dy))
    nrc = int(L.load().ewvit_dwconv3x3_bn_rows(N, H, W, C, 1, 1))
    assert nrc == (N * H + 31) // 32
    part = torch.full((nrc, 2 * C), float('nan'), device=DEV)
    L.call('ewvit_dwconv3x3_bwd_data_bn', L.ptr(dy), L.ptr(w), L.ptr(dx1), N, H, W, C, L.ptr(bx), L.ptr(mean),
           L.ptr(invstd), L.ptr(gamma), L.ptr(beta), 2, L.ptr(part), L.stream(dy))
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    ra, rb, ma, mb = _bwd_ref(dx1, bx, mean, invstd, gamma, beta, 2)
    ea, eb = sums_close(part, ra, rb, ma, mb)
    assert ea < 1e-5 and eb < 1e-5, (ea, eb)


@pytest.mark.parametrize('N,C,H,W,act', [(64, 1536, 7, 7, 2), (64, 960, 14, 14, 2), (4, 200, 9, 11, 2),
                                         (2, 64, 30, 30, 1), (3, 40, 1, 5, 0), (2, 48, 2, 1, 2)])
def test_dw_bwd_fused(N, C, H, W, act):
    """ewvit_dwconv3x3_bwd_fused (dx + the producing BN's backward sums + dW in one pass) against
    the two kernels it replaces: dx bit-exact (same tap order), the BN sums as
    test_dw_bwd_data_bn, dW within 1e-5 of its largest entry (fp32, other summation order);
    accumulate = 1 adds into dW."""
    L = _L()
    g = torch.Generator().manual_seed(C * 5 + W)
    dy = bf(torch.randn(N, C, H, W, generator=g))
    x = bf(torch.randn(N, C, H, W, generator=g))
    bx = bf(torch.randn(N, C, H, W, generator=g) * 1.5 + 0.3)
    w = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).to(DEV).contiguous()
    gamma = (torch.randn(C, generator=g) * 0.3 + 1).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV)
    mean, invstd = _bn_stats(bx)
    dx0, dx1 = torch.empty_like(dy), torch.empty_like(dy)
    L.call('ewvit_dwconv3x3_bwd_data', L.ptr(dy), L.ptr(w), L.ptr(dx0), N, H, W, C, 1, 1, L.BF16, L.stream(dy))
    ws0 = torch.empty(int(L.load().ewvit_dwconv3x3_bwd_weight_workspace(N, H, W, C, 1, 1)) // 4, device=DEV)
    dw0 = torch.empty(C, 1, 3, 3, device=DEV)
    L.call('ewvit_dwconv3x3_bwd_weight', L.ptr(x), L.ptr(dy), L.ptr(dw0), 0, N, H, W, C, 1, 1, L.BF16, L.ptr(ws0),
           L.stream(dy))
    nrc = int(L.load().ewvit_dwconv3x3_bn_rows(N, H, W, C, 1, 1))
    part = torch.full((nrc, 2 * C), float('nan'), device=DEV)
    wsb = int(L.load().ewvit_dwconv3x3_bwd_fused_workspace(N, H, W, C))
    assert wsb == nrc * C * 9 * 4
    ws = torch.full((wsb // 4,), float('nan'), device=DEV)
    dw1 = torch.full((C, 1, 3, 3), float('nan'), device=DEV)
    L.call('ewvit_dwconv3x3_bwd_fused', L.ptr(dy), L.ptr(w), L.ptr(dx1), L.ptr(x), L.ptr(dw1), 0, N, H, W, C,
           L.ptr(bx), L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), act, L.ptr(part), L.ptr(ws), L.stream(dy))
    dwa = torch.full((C, 1, 3, 3), 0.5, device=DEV)
    part2 = torch.empty_like(part)
    L.call('ewvit_dwconv3x3_bwd_fused', L.ptr(dy), L.ptr(w), L.ptr(dx1), L.ptr(x), L.ptr(dwa), 1, N, H, W, C,
           L.ptr(bx), L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), act, L.ptr(part2), L.ptr(ws), L.stream(dy))
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    ra, rb, ma, mb = _bwd_ref(dx1, bx, mean, invstd, gamma, beta, act)
    ea, eb = sums_close(part, ra, rb, ma, mb)
    assert ea < 1e-5 and eb < 1e-5, (ea, eb)
    assert torch.equal(part, part2)
    ref = torch.zeros(C, 9, dtype=torch.float64)
    xp = torch.nn.functional.pad(x.double().cpu(), (1, 1, 1, 1))
    dyd = dy.double().cpu()
    for kh in range(3):
        for kw in range(3):
            ref[:, kh * 3 + kw] = (dyd * xp[:, :, kh:kh + H, kw:kw + W]).sum((0, 2, 3))
    ref = ref.view(C, 1, 3, 3).float().to(DEV)
    scale = float(ref.abs().max())
    assert not torch.isnan(dw1).any()
    assert float((dw1 - ref).abs().max()) / scale < 1e-5
    assert float((dw1 - dw0).abs().max()) / scale < 1e-5
    assert float((dwa - 0.5 - dw1).abs().max()) / scale < 1e-6


@pytest.mark.parametrize('N,H,W,Cin,Cout,act,addend,scaled', [
    (64, 7, 7, 256, 1536, 0, True, True),      # stage-6 expand dgrad + skip: the project BN of the block before
    (64, 14, 14, 160, 960, 0, True, True),     # stage 5 (Ncol 160: a half-empty column tile)
    (64, 7, 7, 256, 1280, 0, False, True),     # the head conv's dgrad: the last block's tail
    (64, 14, 14, 128, 768, 0, False, False),   # a non-residual tail (BatchNorm, no activation)
    (16, 14, 14, 64, 256, 2, False, False),    # a BN + SiLU before a 1x1 conv
])
def test_conv_dgrad_bn(N, H, W, Cin, Cout, act, addend, scaled):
    L = _L()
    g = torch.Generator().manual_seed(Cin + Cout)
    dy = bf(torch.randn(N, Cout, H, W, generator=g))
    wt = torch.randn(Cout, Cin, 1, 1, generator=g) * 0.05
    wpt = wt.reshape(Cout, Cin).t().contiguous().to(DEV, torch.bfloat16)      # [Cin][1][Cout]
    bx = bf(torch.randn(N, Cin, H, W, generator=g) * 1.2 - 0.1)
    gamma = (torch.randn(Cin, generator=g) * 0.3 + 1).to(DEV)
    beta = (torch.randn(Cin, generator=g) * 0.2).to(DEV)
    mean, invstd = _bn_stats(bx)
    sk = bf(torch.randn(N, Cin, H, W, generator=g)) if addend else None
    rs = ((torch.rand(N, generator=g) < 0.8).float() / 0.8).to(DEV) if scaled else None
    dx0, dx1 = torch.empty_like(bx), torch.empty_like(bx)
    if addend:
        L.call('ewvit_conv2d_bwd_data_add', L.ptr(dy), L.ptr(wpt), L.ptr(dx0), L.ptr(sk), N, H, W, Cin, Cout, 1, 1,
               L.stream(dy))
    else:
        L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx0), N, H, W, Cin, Cout, 1, 1, 0, 0,
               L.stream(dy))
    rows = int(L.load().ewvit_conv2d_bwd_bn_rows(N, H, W, Cin, Cout, 1, 1))
    assert rows in ((N * H * W + 127) // 128, (N * H * W + 63) // 64)     # 64-row tiles on small grids
    part = torch.full((rows, 2 * Cin), float('nan'), device=DEV)
    nrc = ctypes.c_int(0)
    L.call('ewvit_conv2d_bwd_data_bn', L.ptr(dy), L.ptr(wpt), L.ptr(dx1), L.ptr(sk), N, H, W, Cin, Cout, 1, 1, 0, 0,
           L.ptr(bx), L.ptr(mean), L.ptr(invstd), L.ptr(gamma if act else None), L.ptr(beta if act else None), act,
           L.ptr(rs), 0, L.ptr(part), ctypes.byref(nrc), L.stream(dy))
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    assert 1 <= nrc.value <= rows
    ra, rb, ma, mb = _bwd_ref(dx1, bx, mean, invstd, gamma, beta, act, rs)
    ea, eb = sums_close(part[:nrc.value], ra, rb, ma, mb)
    assert ea < 1e-5 and eb < 1e-5, (ea, eb)


@pytest.mark.parametrize('act,scaled', [(2, False), (0, True), (0, False)])
def test_bn_bwd_partials_matches_reduce(act, scaled):
    """ewvit_bn_bwd_partials from a producer's partial rows == ewvit_bn_bwd(_scaled) (which
    sums the same terms itself), to the fp32 summation order."""
    L = _L()
    N, C, H, W = 32, 512, 14, 14
    M = N * H * W
    g = torch.Generator().manual_seed(act + 10 * scaled)
    dy = bf(torch.randn(N, C, H, W, generator=g))
    bx = bf(torch.randn(N, C, H, W, generator=g) + 0.2)
    gamma = (torch.randn(C, generator=g) * 0.3 + 1).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV)
    mean, invstd = _bn_stats(bx)
    rs = ((torch.rand(N, generator=g) < 0.75).float() / 0.75).to(DEV) if scaled else None
    ra, rb, _, _ = _bwd_ref(dy, bx, mean, invstd, gamma, beta, act, rs)
    part = torch.stack([ra, rb]).reshape(1, 2 * C).float().to(DEV)     # one exact partial row
    dx0, dx1 = torch.empty_like(dy), torch.empty_like(dy)
    dg0, db0, dg1, db1 = (torch.empty(C, device=DEV) for _ in range(4))
    ws = torch.empty(L.load().ewvit_bn_workspace(M, C, 1) // 4, device=DEV)
    if scaled:
        L.call('ewvit_bn_bwd_scaled', L.ptr(dy), L.ptr(bx), L.ptr(dx0), L.BF16, M, C, L.ptr(gamma), L.ptr(beta),
               L.ptr(mean), L.ptr(invstd), L.ptr(dg0), L.ptr(db0), L.ptr(rs), H * W, L.ptr(ws), L.stream(dy))
    else:
        L.call('ewvit_bn_bwd', L.ptr(dy), L.ptr(bx), L.ptr(dx0), L.BF16, M, C, L.ptr(gamma), L.ptr(beta), L.ptr(mean),
               L.ptr(invstd), act, L.ptr(dg0), L.ptr(db0), 0, 1, L.ptr(ws), L.stream(dy))
    L.call('ewvit_bn_bwd_partials', L.ptr(dy), L.ptr(bx), L.ptr(dx1), L.BF16, M, C, L.ptr(gamma), L.ptr(beta),
           L.ptr(mean), L.ptr(invstd), act, L.ptr(dg1), L.ptr(db1), L.ptr(rs), H * W, L.ptr(part), 1, 1, L.stream(dy))
    torch.cuda.synchronize()
    d = (dx0.float() - dx1.float()).abs()
    assert float(d.max()) <= 2 ** -6 * float(dx0.float().abs().max()), float(d.max())
    assert float((d > 0).float().mean()) < 0.02
    for a, b in ((dg0, dg1), (db0, db1)):
        assert float((a - b).abs().max()) <= 1e-5 * float(a.abs().max()) + 1e-6


def _run(mods, x0, dyo, linked, monkeypatch):
    import ewvit
    import ewvit.bn as ebn
    import network.efficientnet as en
    L = ewvit._lib
    monkeypatch.setattr(ebn, '_BWD_LINK', linked)
    monkeypatch.setattr(en, '_DW_STATS', linked)
    m = mods().to(DEV).to(memory_format=torch.channels_last).train()
    for mod in m.modules():
        if hasattr(mod, 'sd_prob'):
            mod.sd_prob = 0.0          # no drop-path draw: both runs see the same keep masks
    x = x0.clone().requires_grad_(True)
    calls = {}
    real = L.call

    def count(name, *a, **k):
        calls[name] = calls.get(name, 0) + 1
        return real(name, *a, **k)
    monkeypatch.setattr(L, 'call', count)
    try:
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y = m(x)
        y.backward(dyo)
    finally:
        monkeypatch.setattr(L, 'call', real)
    torch.cuda.synchronize()
    return (y.detach().float(), x.grad.float(), {n: p.grad.float() for n, p in m.named_parameters()},
            {n: b.float() for n, b in m.named_buffers() if 'running' in n}, calls)


def _features(sl):
    def make():
        from network.efficientnet import EfficientNetV2S
        torch.manual_seed(1)
        f = EfficientNetV2S().features
        return torch.nn.Sequential(*[f[s][b] for s, b in sl])
    return make


def _cos(a, b):
    return float(torch.nn.functional.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0))


def test_mbconv_blocks_linked_vs_unlinked(monkeypatch):
    """Four MBConv blocks (5.7, 5.8 at 14^2, the stride-2 6.0, 6.1 at 7^2) train step with the
    BN links on and off: the same numbers to fp32 summation order (a short chain, so bf16
    rounding differences cannot compound much), and the linked run launched the fused kernels.
    Measured (tools/diag_link.py): the forward drifts only through the depthwise BN statistics
    (other fp32 summation order), 1 - cos = 1e-8 after one block, 7e-7 after two, 2.4e-5 after
    four — the amplification any two bf16 runs of this random-init stack show; the backward
    links alone leave the forward bit-identical (input-gradient cosine 0.99999)."""
    g = torch.Generator().manual_seed(5)
    N = 32
    x0 = torch.randn(N, 160, 14, 14, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dyo = torch.randn(N, 256, 7, 7, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    mods = _features([(5, 7), (5, 8), (6, 0), (6, 1)])
    y0, gx0, gp0, bf0, c0 = _run(mods, x0, dyo, False, monkeypatch)
    y1, gx1, gp1, bf1, c1 = _run(mods, x0, dyo, True, monkeypatch)
    assert c0.get('ewvit_bn_bwd_partials', 0) == 0
    assert c1.get('ewvit_dwconv3x3_fwd_bn', 0) == 4
    # 6.0's depthwise is stride 2; the stride-1 ones take dx, the link and dW in one pass
    assert c1.get('ewvit_dwconv3x3_bwd_fused', 0) == 3 and c1.get('ewvit_dwconv3x3_bwd_data_bn', 0) == 0
    assert c1.get('ewvit_dwconv3x3_bwd_weight', 0) == 1 and c0.get('ewvit_dwconv3x3_bwd_weight', 0) == 4
    # the tails of 5.7, 5.8, 6.0
    assert c1.get('ewvit_conv2d_bwd_data_bn', 0) == 3
    assert c1.get('ewvit_bn_bwd_partials', 0) == 6
    assert _cos(y0, y1) > 0.9999 and float((y0 - y1).abs().max()) <= 5e-2 * float(y0.abs().max())
    assert _cos(gx0, gx1) > 0.9995
    # a BatchNorm bias whose output gradient passes only through train-mode BatchNorms (and
    # skips of them) has an exactly zero true gradient — its computed one is rounding noise in
    # both runs (cosine ~0.1): biases are held to an absolute bound instead
    worst = min((_cos(gp0[n], gp1[n]), n) for n in gp0 if gp0[n].abs().max() > 0 and not n.endswith('bias'))
    assert worst[0] > 0.995, worst
    top = max(float(v.abs().max()) for v in gp0.values())
    for n in gp0:
        if n.endswith('bias'):
            assert float((gp0[n] - gp1[n]).abs().max()) <= 1e-2 * top, n
    # running statistics after one update (0.9 * init + 0.1 * batch): 1e-3 relative, or 2e-4
    # absolute for a mean that is itself a near-zero cancellation (a project conv's output)
    for n in bf0:
        assert float((bf0[n] - bf1[n]).abs().max()) <= 1e-3 * float(bf0[n].abs().max()) + 2e-4, n


def test_mbconv_stages_link_count(monkeypatch):
    """Stages 4-6 (all 30 MBConv blocks): every BN the links can serve is served — the
    depthwise BNs' statistics in the conv, each stride-1 block's expand-BN reduction in its
    depthwise input gradient, each tail's reduction in the next block's first input gradient —
    and the step stays finite (the numbers are compared on the short chain above; over 30
    blocks two bf16 implementations drift apart like any two bf16 runs)."""
    g = torch.Generator().manual_seed(9)
    N = 16
    x0 = torch.randn(N, 64, 28, 28, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dyo = torch.randn(N, 256, 7, 7, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    sl = [(4, b) for b in range(6)] + [(5, b) for b in range(9)] + [(6, b) for b in range(15)]
    y1, gx1, gp1, _, c1 = _run(_features(sl), x0, dyo, True, monkeypatch)
    nblk = 30
    assert c1.get('ewvit_dwconv3x3_fwd_bn', 0) == nblk
    assert c1.get('ewvit_dwconv3x3_bwd_fused', 0) == nblk - 2            # blocks 4.0 / 6.0 are stride 2
    assert c1.get('ewvit_dwconv3x3_bwd_weight', 0) == 2
    # the last tail has no conv after it
    assert c1.get('ewvit_conv2d_bwd_data_bn', 0) == nblk - 1
    assert c1.get('ewvit_bn_bwd_partials', 0) == 2 * nblk - 3
    nbwd = c1.get('ewvit_bn_bwd', 0) + c1.get('ewvit_bn_bwd_scaled', 0) + c1.get('ewvit_bn_bwd_partials', 0)
    assert nbwd == 2 * nblk, c1
    assert c1.get('ewvit_bn_bwd', 0) == 2 and c1.get('ewvit_bn_bwd_scaled', 0) == 1
    assert bool(torch.isfinite(y1).all()) and bool(torch.isfinite(gx1).all())
    assert all(bool(torch.isfinite(v).all()) for v in gp1.values())


@pytest.mark.parametrize('N,C,H', [(32, 960, 14), (32, 1536, 7)])
def test_dw_stats_bn_act_se_matches(N, C, H, monkeypatch):
    """One depthwise conv + BN + SiLU + SE (ewvit.bn_act_se) with the statistics from the conv
    kernel vs from the BN's own statistics pass: same batch statistics to fp32 rounding, same
    outputs up to the bf16 rounding those last bits can flip."""
    import ewvit
    from network.efficientnet import ConvBNAct, SqueezeExcitation
    torch.manual_seed(C)
    blk = ConvBNAct(C, C, 3, 1, groups=C).to(DEV).train()
    se = SqueezeExcitation(C, C // 24).to(DEV)
    x = (torch.randn(N, C, H, H) * 0.8 + 0.3).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for linked in (False, True):
        rm0, rv0 = blk[1].running_mean.clone(), blk[1].running_var.clone()
        r = blk.dw_stats(x) if linked else None
        if linked:
            assert r is not None
        y = r[0] if linked else blk[0](x)
        o = ewvit.bn_act_se(y, blk[1], 'silu', se.fc1.weight, se.fc1.bias, se.fc2.weight, se.fc2.bias,
                            partials=r[1:] if linked else None)
        outs.append((y, o, blk[1].running_mean.clone(), blk[1].running_var.clone()))
        blk[1].running_mean.copy_(rm0)
        blk[1].running_var.copy_(rv0)
    (y0, o0, m0, v0), (y1, o1, m1, v1) = outs
    assert torch.equal(y0, y1)
    assert float((m0 - m1).abs().max()) <= 1e-6 * float(m0.abs().max()) + 1e-7
    assert float((v0 - v1).abs().max()) <= 1e-5 * float(v0.abs().max())
    d = (o0.float() - o1.float()).abs()
    assert float((d > 0).float().mean()) < 0.01, float((d > 0).float().mean())
    assert float(d.max()) <= 2 ** -7 * float(o0.float().abs().max())


def _wpack_t(w):
    """[Cout][Cin][k][k] fp32 -> the bwd_data pack [Cin][k*k][Cout] bf16 (ewvit_conv2d_pack_weight)."""
    Cout, Cin, k, _ = w.shape
    return w.permute(1, 2, 3, 0).reshape(Cin, k * k, Cout).contiguous().to(DEV, torch.bfloat16)


@pytest.mark.parametrize('cap', [0, 24])
def test_conv_dgrad_bn_channel_groups(cap):
    """The multiscale_fusion shape class: a level-major input read as its channel concatenation
    (grouped dx), one BatchNorm group per level (the fusion BN's per-level statistics), the MWT
    under a workgroup cap (persistent walk): dx bit-identical to ewvit_conv2d_bwd_data, each
    level's partial rows = fp64 sums of its own g terms."""
    L = _L()
    lib = L.load()
    Lv, N, C, Cout, H, W = 3, 2, 128, 128, 20, 18
    g = torch.Generator().manual_seed(11)
    dy = bf(torch.randn(N, Cout, H, W, generator=g))
    w = torch.randn(Cout, Lv * C, 3, 3, generator=g) / (9 * Lv * C) ** 0.5
    wpt = _wpack_t(w)
    bxz = bf(torch.randn(Lv * N, C, H, W, generator=g) + 0.2)           # level-major BN input
    mean = torch.stack([bxz[l * N:(l + 1) * N].float().mean((0, 2, 3)) for l in range(Lv)]).contiguous()
    invstd = torch.stack([torch.rsqrt(bxz[l * N:(l + 1) * N].float().var((0, 2, 3), unbiased=False) + 1e-5)
                          for l in range(Lv)]).contiguous()
    gamma = (torch.randn(C, generator=g) * 0.3 + 1).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV)
    gs = N * H * W * C
    dx0, dx1 = torch.empty_like(bxz), torch.empty_like(bxz)
    prev = lib.ewvit_set_grid_cap(cap)
    try:
        L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx0), N, H, W, Lv * C, Cout, 3, 1, C, gs,
               L.stream(dy))
        tiles = int(lib.ewvit_conv2d_bwd_bn_rows(N, H, W, Lv * C, Cout, 3, 1))
        assert tiles in ((N * H * W + 127) // 128, (N * H * W + 63) // 64)
        part = torch.full((Lv * tiles, 2 * C), float('nan'), device=DEV)
        nrc = ctypes.c_int(0)
        L.call('ewvit_conv2d_bwd_data_bn', L.ptr(dy), L.ptr(wpt), L.ptr(dx1), None, N, H, W, Lv * C, Cout, 3, 1, C,
               gs, L.ptr(bxz), L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), 1, None, 0, L.ptr(part),
               ctypes.byref(nrc), L.stream(dy))
    finally:
        lib.ewvit_set_grid_cap(prev)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    assert nrc.value == tiles
    for lv in range(Lv):
        sl = slice(lv * N, (lv + 1) * N)
        # ReLU: g = dx where the BN output is positive
        d, x = dx1[sl].double().cpu(), bxz[sl].double().cpu()
        xh = (x - mean[lv].double().cpu().view(1, C, 1, 1)) * invstd[lv].double().cpu().view(1, C, 1, 1)
        z = xh * gamma.double().cpu().view(1, C, 1, 1) + beta.double().cpu().view(1, C, 1, 1)
        gr = torch.where(z > 0, d, torch.zeros_like(d))
        ra, rb = gr.sum((0, 2, 3)), (gr * xh).sum((0, 2, 3))
        ma, mb = gr.abs().sum((0, 2, 3)), (gr * xh).abs().sum((0, 2, 3))
        ea, eb = sums_close(part[lv * tiles:(lv + 1) * tiles], ra, rb, ma, mb)
        assert ea < 1e-5 and eb < 1e-5, (lv, ea, eb)


@pytest.mark.parametrize('cap', [0, 16])
def test_conv_dgrad_bn_row_groups(cap):
    """The hf_conv fusion shape class: a plain input whose BatchNorm has one statistics group
    per level (consecutive batch slices, mean / invstd [groups][C]): partial rows grouped by
    level, each = fp64 sums of its slice's g terms; dx bit-identical; capped walk too."""
    L = _L()
    lib = L.load()
    Lv, N, C, Cout, H, W = 3, 2, 64, 128, 16, 16       # N*H*W = 512 rows per level (4 m-tiles)
    g = torch.Generator().manual_seed(12)
    dy = bf(torch.randn(Lv * N, Cout, H, W, generator=g))
    w = torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5
    wpt = _wpack_t(w)
    bx = bf(torch.randn(Lv * N, C, H, W, generator=g) * 0.7 + 0.1)
    mean = torch.stack([bx[l * N:(l + 1) * N].float().mean((0, 2, 3)) for l in range(Lv)]).contiguous()
    invstd = torch.stack([torch.rsqrt(bx[l * N:(l + 1) * N].float().var((0, 2, 3), unbiased=False) + 1e-5)
                          for l in range(Lv)]).contiguous()
    gamma = (torch.randn(C, generator=g) * 0.3 + 1).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV)
    dx0, dx1 = torch.empty_like(bx), torch.empty_like(bx)
    M = Lv * N * H * W
    prev = lib.ewvit_set_grid_cap(cap)
    # (the plain dgrad of this 64-column shape would take the windowed k-split kernel, whose k
    # order differs: the generic LDS-DMA kernel is the bit-identity reference here)
    lib.ewvit_conv2d_set_win(0)
    try:
        L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx0), Lv * N, H, W, C, Cout, 3, 1, 0, 0,
               L.stream(dy))
        lib.ewvit_conv2d_set_win(1)
        tiles = int(lib.ewvit_conv2d_bwd_bn_rows(Lv * N, H, W, C, Cout, 3, 1))
        part = torch.full((tiles, 2 * C), float('nan'), device=DEV)
        nrc = ctypes.c_int(0)
        L.call('ewvit_conv2d_bwd_data_bn', L.ptr(dy), L.ptr(wpt), L.ptr(dx1), None, Lv * N, H, W, C, Cout, 3, 1, 0,
               0, L.ptr(bx), L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), 1, None, M // Lv, L.ptr(part),
               ctypes.byref(nrc), L.stream(dy))
    finally:
        lib.ewvit_set_grid_cap(prev)
        lib.ewvit_conv2d_set_win(1)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    per = tiles // Lv                                  # 128-row tiles, or 64 on small grids
    assert nrc.value == per and tiles == Lv * per and per in (M // Lv // 128, M // Lv // 64)
    for lv in range(Lv):
        sl = slice(lv * N, (lv + 1) * N)
        d, x = dx1[sl].double().cpu(), bx[sl].double().cpu()
        xh = (x - mean[lv].double().cpu().view(1, C, 1, 1)) * invstd[lv].double().cpu().view(1, C, 1, 1)
        z = xh * gamma.double().cpu().view(1, C, 1, 1) + beta.double().cpu().view(1, C, 1, 1)
        gr = torch.where(z > 0, d, torch.zeros_like(d))
        ea, eb = sums_close(part[lv * per:(lv + 1) * per], gr.sum((0, 2, 3)), (gr * xh).sum((0, 2, 3)),
                            gr.abs().sum((0, 2, 3)), (gr * xh).abs().sum((0, 2, 3)))
        assert ea < 1e-5 and eb < 1e-5, (lv, ea, eb)


def test_stale_offer_not_taken():
    """A BatchNorm's link offer dies with its output: a later tensor at the same address and
    shape (the caching allocator reuses blocks) does not pick it up."""
    import ewvit.bn as ebn
    y = torch.empty(2, 8, 4, 4, dtype=torch.bfloat16, device=DEV)
    x = torch.empty_like(y)
    m = torch.zeros(1, 8, device=DEV)
    ebn.offer_bwd_link(y, x, m, m, None, None, 0)
    key = ebn._tls.offered.key
    del y
    z = torch.empty(2, 8, 4, 4, dtype=torch.bfloat16, device=DEV)
    if (z.data_ptr(), tuple(z.shape), z.dtype) == key:
        assert ebn.take_bwd_link(z) is None
    ebn._tls.offered = None


@pytest.mark.parametrize('kind', ['grouped', 'drop_add'])
def test_dwconv_refuses_links_it_cannot_sum(kind, monkeypatch):
    """ewvit_dwconv3x3_bwd_data_bn leaves whole-map, unscaled backward sums, so the
    depthwise conv must not take the link of a grouped BatchNorm (per-level statistics, e.g.
    the MWT's) nor of a BNDropAdd tail (drop-path row scale): with the links on, the gradients
    equal the EWVIT_BN_BWD_LINK=0 ones (the BN's own reduction pass runs)."""
    import ewvit
    import ewvit.bn as ebn
    g = torch.Generator().manual_seed(21)
    N, C, H = 8, 64, 14
    x = (torch.randn(N, C, H, H, generator=g) * 0.7 + 0.2).to(DEV, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    skip = torch.randn(N, C, H, H, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wdw = (torch.randn(C, 1, 3, 3, generator=g) / 3).to(DEV)
    dyo = torch.randn(N, C, H, H, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for linked in (False, True):
        monkeypatch.setattr(ebn, '_BWD_LINK', linked)
        torch.manual_seed(4)
        bn = torch.nn.BatchNorm2d(C).to(DEV).train()
        xi = x.clone().requires_grad_(True)
        if kind == 'grouped':
            h = ewvit.batch_norm_act(xi, bn, 'silu', groups=2)
        else:
            h = ewvit.bn.batch_norm_drop_add(xi, bn, skip, 0.5)
        y = ewvit.dwconv3x3(h, wdw.requires_grad_(True))
        y.backward(dyo)
        torch.cuda.synchronize()
        res.append((xi.grad.float(), bn.weight.grad.clone(), bn.bias.grad.clone()))
        wdw = wdw.detach()
    for a, b in zip(*res):
        torch.testing.assert_close(b, a, rtol=0, atol=0)


@pytest.mark.parametrize('N,C,H,W,act', [(64, 960, 14, 14, 2), (16, 1536, 7, 7, 2), (4, 200, 9, 11, 1), (2, 64, 30, 30, 0)])
def test_dw_bwd_fused_se(N, C, H, W, act):
    """ewvit_dwconv3x3_bwd_fused_se (the BN(+act) + SE backward of the conv's output folded into
    the fused depthwise backward: dz formed per window element from the SE output gradient and z)
    against ewvit_bn_se_bwd_dx (that dx pass alone, writing dz) + ewvit_dwconv3x3_bwd_fused on dz:
    dx, the producing BN's backward sums and dW bit for bit with act 0 / 1; with SiLU (act 2) the
    compiler schedules the exp / reciprocal differently in the two kernels, so dz may differ by one
    bf16 rounding: dx within 2 bf16 ulps of its scale, the sums and dW within 1e-3 relative."""
    L = _L()
    g = torch.Generator().manual_seed(C * 7 + W)
    dys = bf(torch.randn(N, C, H, W, generator=g))
    z = bf(torch.randn(N, C, H, W, generator=g) * 1.3 - 0.2)
    x = bf(torch.randn(N, C, H, W, generator=g))
    bx = bf(torch.randn(N, C, H, W, generator=g) * 1.5 + 0.3)
    w = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).to(DEV).contiguous()
    gamma = (torch.randn(C, generator=g) * 0.3 + 1).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV)
    g2 = (torch.randn(C, generator=g) * 0.3 + 1).to(DEV)
    b2 = (torch.randn(C, generator=g) * 0.2).to(DEV)
    mean, invstd = _bn_stats(bx)
    m2, i2 = _bn_stats(z)
    s = torch.rand(N, C, generator=g).to(DEV)
    gs = (torch.randn(N, C, generator=g) * 0.01).to(DEV)
    row = (torch.randn(2 * C, generator=g) * N * H * W * 0.01).to(DEV)
    dz = torch.empty_like(dys)
    L.call('ewvit_bn_se_bwd_dx', L.ptr(dys), L.ptr(z), L.ptr(dz), L.BF16, N, H * W, C, L.ptr(g2), L.ptr(b2), L.ptr(m2),
           L.ptr(i2), act, L.ptr(s), L.ptr(gs), L.ptr(row), L.stream(dys))
    nrc = int(L.load().ewvit_dwconv3x3_bn_rows(N, H, W, C, 1, 1))
    wsb = int(L.load().ewvit_dwconv3x3_bwd_fused_workspace(N, H, W, C))
    outs = []
    for fold in (False, True):
        dx = torch.full_like(dys, float('nan'))
        part = torch.full((nrc, 2 * C), float('nan'), device=DEV)
        ws = torch.full((wsb // 4,), float('nan'), device=DEV)
        dw = torch.full((C, 1, 3, 3), float('nan'), device=DEV)
        if fold:
            L.call('ewvit_dwconv3x3_bwd_fused_se', L.ptr(dys), L.ptr(w), L.ptr(dx), L.ptr(x), L.ptr(dw), 0, N, H, W, C,
                   L.ptr(bx), L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), 2, L.ptr(part), L.ptr(ws),
                   L.ptr(z), L.ptr(m2), L.ptr(i2), L.ptr(g2), L.ptr(b2), act, L.ptr(row), L.ptr(s), L.ptr(gs),
                   L.stream(dys))
        else:
            L.call('ewvit_dwconv3x3_bwd_fused', L.ptr(dz), L.ptr(w), L.ptr(dx), L.ptr(x), L.ptr(dw), 0, N, H, W, C,
                   L.ptr(bx), L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), 2, L.ptr(part), L.ptr(ws),
                   L.stream(dys))
        outs.append((dx, part, dw))
    torch.cuda.synchronize()
    (dx0, p0, w0), (dx1, p1, w1) = outs
    assert not torch.isnan(dx1).any() and not torch.isnan(w1).any()
    if act != 2:
        assert torch.equal(dx0, dx1), float((dx0.float() - dx1.float()).abs().max())
        assert torch.equal(p0, p1)
        assert torch.equal(w0, w1)
        return
    sc = float(dx0.float().abs().max())
    assert float((dx0.float() - dx1.float()).abs().max()) <= 2 * sc * 2 ** -8
    for a, b in ((p0, p1), (w0, w1)):
        assert float((a - b).abs().max()) <= 1e-3 * float(a.abs().max())
