"""Squeeze-excitation and stochastic-depth residual kernels (csrc/se.hip) through
the C-ABI, vs torch fp32 on the same (bf16-rounded) inputs.

Tolerance: bf16 outputs are one rounding of an fp32 result (2^-7 of scale); f32
outputs 1e-5; gradients 2e-3 of scale (fp32 reductions in another order) and
2e-2 for bf16 input gradients (one bf16 rounding of dy*s + g).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


def ref_se(x, w1, b1, w2, b2):
    s = x.mean((2, 3), keepdim=True)
    s = torch.sigmoid(F.conv2d(F.silu(F.conv2d(s, w1, b1)), w2, b2))
    return x * s


@pytest.mark.parametrize('N,C,H,W,csq', [(4, 256, 28, 28, 16), (3, 960, 14, 14, 40), (2, 1536, 7, 7, 64),
                                         (5, 24, 9, 11, 6), (2, 2048, 3, 3, 8), (64, 960, 14, 14, 40)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_squeeze_excite(N, C, H, W, csq, dtype):
    import ewvit
    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(N, C, H, W, generator=g).to(dtype)
    w1 = torch.randn(csq, C, 1, 1, generator=g) / C ** 0.5
    b1 = torch.randn(csq, generator=g) * 0.1
    w2 = torch.randn(C, csq, 1, 1, generator=g) / csq ** 0.5
    b2 = torch.randn(C, generator=g) * 0.1
    ps = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
    xr = x.float().clone().requires_grad_(True)
    yr = ref_se(xr, *ps)
    dy = torch.randn(yr.shape, generator=g).to(dtype)
    yr.backward(dy.float())
    xd = x.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    pd = [t.to(DEV).to(memory_format=torch.channels_last) if t.dim() == 4 else t.to(DEV) for t in (w1, b1, w2, b2)]
    pd = [t.requires_grad_(True) for t in pd]
    y = ewvit.squeeze_excite(xd, *pd)
    y.backward(dy.to(DEV).to(memory_format=torch.channels_last))
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    assert rel(y, yr) < (2 ** -7 if dtype == torch.bfloat16 else 1e-5)
    assert rel(xd.grad, xr.grad) < (2e-2 if dtype == torch.bfloat16 else 2e-4)
    for a, b in zip(pd, ps):
        assert a.grad.shape == b.shape and a.grad.stride() == a.stride()
        assert rel(a.grad, b.grad) < 2e-3


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_scale_add(dtype):
    import ewvit
    g = torch.Generator().manual_seed(9)
    r = torch.randn(6, 64, 7, 9, generator=g).to(dtype)
    x = torch.randn(6, 64, 7, 9, generator=g).to(dtype)
    keep = torch.tensor([1., 0., 1., 1., 0., 1.]) / 0.8
    rr, xr = r.float().clone().requires_grad_(True), x.float().clone().requires_grad_(True)
    yr = rr * keep.view(-1, 1, 1, 1) + xr
    dy = torch.randn(yr.shape, generator=g).to(dtype)
    yr.backward(dy.float())
    rd = r.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    xd = x.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    y = ewvit.scale_add(rd, keep.to(DEV), xd)
    y.backward(dy.to(DEV).to(memory_format=torch.channels_last))
    tol = 2 ** -7 if dtype == torch.bfloat16 else 1e-6
    assert rel(y, yr) < tol
    assert rel(rd.grad, rr.grad) < tol and rel(xd.grad, xr.grad) < tol


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_drop_add(dtype):
    """StochasticDepth(row) + skip add with the keep mask drawn in-kernel: y and the
    gradients follow r * scale[n] + x for the 0 / 1/keep factors the kernel drew;
    the kept fraction matches keep over many rows; a new step counter redraws."""
    import ewvit
    from ewvit import _lib as L
    g = torch.Generator().manual_seed(10)
    N, p = 4096, 0.3
    r = torch.randn(N, 16, 3, 3, generator=g).to(dtype).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(N, 16, 3, 3, generator=g).to(dtype).to(DEV).to(memory_format=torch.channels_last)
    rd, xd = r.clone().requires_grad_(True), x.clone().requires_grad_(True)
    y = ewvit.drop_add(rd, xd, p)
    dy = torch.randn(y.shape, generator=g).to(dtype).to(DEV).to(memory_format=torch.channels_last)
    y.backward(dy)
    # recover the factors from the rows: kept rows have y - x = r / (1-p)
    kept = ((y.float() - x.float()).abs().flatten(1).amax(1) > 0)
    sc = kept.float() / (1 - p)
    yr = r.float() * sc.view(-1, 1, 1, 1) + x.float()
    tol = 2 ** -7 if dtype == torch.bfloat16 else 1e-6
    assert rel(y, yr) < tol
    assert rel(rd.grad, dy.float() * sc.view(-1, 1, 1, 1)) < tol and rel(xd.grad, dy) < tol
    frac = float(kept.float().mean())
    assert abs(frac - (1 - p)) < 4 * ((p * (1 - p) / N) ** 0.5)
    L.rng_advance(r.device)
    with torch.no_grad():
        y2 = ewvit.drop_add(r, x, p)
    kept2 = ((y2.float() - x.float()).abs().flatten(1).amax(1) > 0)
    assert not torch.equal(kept, kept2)


@pytest.mark.parametrize('kind,hw', [('mb', 7), ('mb', 14), ('fused', 12)])
def test_block_tail_bn_drop_add(kind, hw, monkeypatch):
    """MBConv / FusedMBConv training forward+backward with the block tail (project BN,
    StochasticDepth, skip add) as one ewvit_bn_fwd_drop_add pass matches the separate
    BN + drop_add path under the same seed (same in-kernel keep mask)."""
    import network.efficientnet as en
    torch.manual_seed(7)
    if kind == 'mb':
        b1, b2 = en.MBConv(6, 3, 1, 64, 64, 0.5), en.MBConv(6, 3, 1, 64, 64, 0.5)
    else:
        b1, b2 = en.FusedMBConv(4, 3, 1, 64, 64, 0.5), en.FusedMBConv(4, 3, 1, 64, 64, 0.5)
    b1, b2 = b1.to(DEV), b2.to(DEV)
    b2.load_state_dict(b1.state_dict())
    x = torch.randn(16, 64, hw, hw, device=DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    torch.manual_seed(11)
    y1 = b1(x1)
    monkeypatch.setattr(en.ConvBNAct, 'can_drop_add', lambda self, x: False)
    torch.manual_seed(11)
    y2 = b2(x2)
    kept = ((y2.float() - x.float()).abs().flatten(1).amax(1) > 0)
    assert 0 < int(kept.sum()) < 16                        # the mask is exercised
    dy = torch.randn(y1.shape, device=DEV).to(torch.bfloat16)
    y1.backward(dy)
    y2.backward(dy)
    assert rel(y1.float(), y2.float()) < 2 ** -6
    assert rel(x1.grad.float(), x2.grad.float()) < 2e-2
    for (n, p1), p2 in zip(b1.named_parameters(), b2.parameters()):
        if p1.grad is not None and p2.grad is not None:
            assert rel(p1.grad, p2.grad) < 3e-2, n
    for (n, q1), q2 in zip(b1.named_buffers(), b2.buffers()):
        assert torch.allclose(q1.float(), q2.float(), rtol=1e-3, atol=1e-5), n


@pytest.mark.parametrize('N,C,H,W,csq', [(64, 1536, 7, 7, 64), (64, 960, 14, 14, 40), (4, 256, 28, 28, 16),
                                         (5, 24, 9, 11, 6)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_bn_act_se(N, C, H, W, csq, dtype):
    """ewvit.bn_act_se = SE(SiLU(BatchNorm(x))) in training mode (MBConv's depthwise BN + SE), its
    backward forming the BN output gradient dy*s + g inside the BN passes: against torch fp32
    BatchNorm2d + SiLU + SE on the same inputs, and the running statistics / counter against
    the module's."""
    import ewvit
    g = torch.Generator().manual_seed(C + W)
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(dtype)
    w1 = torch.randn(csq, C, 1, 1, generator=g) / C ** 0.5
    b1 = torch.randn(csq, generator=g) * 0.1
    w2 = torch.randn(C, csq, 1, 1, generator=g) / csq ** 0.5
    b2 = torch.randn(C, generator=g) * 0.1
    bn_r = torch.nn.BatchNorm2d(C, eps=1e-3).train()
    with torch.no_grad():
        bn_r.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn_r.bias.copy_(torch.randn(C, generator=g) * 0.2)
    bn_d = torch.nn.BatchNorm2d(C, eps=1e-3).train().to(DEV)
    bn_d.load_state_dict(bn_r.state_dict())
    ps = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
    xr = x.float().clone().requires_grad_(True)
    yr = ref_se(F.silu(bn_r(xr)), *ps)
    dy = torch.randn(yr.shape, generator=g).to(dtype)
    yr.backward(dy.float())
    xd = x.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    pd = [t.to(DEV).to(memory_format=torch.channels_last) if t.dim() == 4 else t.to(DEV) for t in (w1, b1, w2, b2)]
    pd = [t.requires_grad_(True) for t in pd]
    y = ewvit.bn_act_se(xd, bn_d, 'silu', *pd)
    y.backward(dy.to(DEV).to(memory_format=torch.channels_last))
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    bf = dtype == torch.bfloat16
    assert rel(y, yr) < (2e-2 if bf else 1e-4)              # bf16: BN output and y each rounded once
    assert rel(xd.grad, xr.grad) < (3e-2 if bf else 5e-4)
    assert rel(bn_d.weight.grad, bn_r.weight.grad) < (2e-2 if bf else 5e-4)
    assert rel(bn_d.bias.grad, bn_r.bias.grad) < (2e-2 if bf else 5e-4)
    for a, b in zip(pd, ps):
        assert a.grad.shape == b.shape
        assert rel(a.grad, b.grad) < (2e-2 if bf else 1e-3)
    assert rel(bn_d.running_mean, bn_r.running_mean) < 1e-3 and rel(bn_d.running_var, bn_r.running_var) < 1e-3
    assert int(bn_d.num_batches_tracked) == int(bn_r.num_batches_tracked) == 1


def test_bn_act_se_matches_two_step_path():
    """bn_act_se against the unfused product path (batch_norm_act, then squeeze_excite): same
    forward bits; the input gradient differs only by the unfused path's bf16 rounding of the SE
    input gradient (dy*s + g)."""
    import ewvit
    g = torch.Generator().manual_seed(4)
    N, C, H, W, csq = 64, 1536, 7, 7, 64
    x = (torch.randn(N, C, H, W, generator=g)).to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    w1 = (torch.randn(csq, C, 1, 1, generator=g) / C ** 0.5).to(DEV)
    b1 = (torch.randn(csq, generator=g) * 0.1).to(DEV)
    w2 = (torch.randn(C, csq, 1, 1, generator=g) / csq ** 0.5).to(DEV)
    b2 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    dy = torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    outs = []
    for fused in (True, False):
        bn = torch.nn.BatchNorm2d(C, eps=1e-3).train().to(DEV)
        xd = x.clone().requires_grad_(True)
        ps = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
        y = ewvit.bn_act_se(xd, bn, 'silu', *ps) if fused else \
            ewvit.squeeze_excite(ewvit.batch_norm_act(xd, bn, 'silu'), *ps)
        y.backward(dy)
        outs.append((y, xd.grad, bn.weight.grad, bn.bias.grad, [p.grad for p in ps], bn.running_var.clone()))
    a, b = outs
    assert torch.equal(a[0], b[0]) and torch.equal(a[5], b[5])
    assert rel(a[1], b[1]) < 1e-2
    assert rel(a[2], b[2]) < 1e-2 and rel(a[3], b[3]) < 1e-2
    # the SE squeeze sum ds = sum_hw dy * a: the fused backward (ewvit_bn_se_bwd) adds its row
    # groups in another (register butterfly) order than the SE-alone pass: fp32 reassociation
    for p, q in zip(a[4], b[4]):
        assert rel(p, q) < 1e-5


@pytest.mark.parametrize('N,C,HW,csq,dtype', [(64, 1536, 49, 64, torch.bfloat16), (64, 960, 196, 40, torch.bfloat16),
                                              (3, 200, 9, 6, torch.bfloat16), (5, 264, 30, 16, torch.float32)])
def test_se_forward_matches_two_launch_path(N, C, HW, csq, dtype):
    """ewvit_se_forward (gates + excite pass in one launch) is bit-identical to
    ewvit_se_squeeze_mlp_fwd + ewvit_se_scale (the same operations in the same order)."""
    import ewvit
    L = ewvit._lib
    g = torch.Generator().manual_seed(C + HW)
    x = torch.randn(N, HW, C, generator=g).to(DEV, dtype)
    w1 = (torch.randn(csq, C, generator=g) / C ** 0.5).to(DEV)
    b1 = (torch.randn(csq, generator=g) * 0.1).to(DEV)
    w2 = (torch.randn(C, csq, generator=g) / csq ** 0.5).to(DEV)
    b2 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    ws = torch.empty(L.load().ewvit_se_mlp_fwd_workspace(N, C, csq) // 4, device=DEV)
    out = []
    for fused in (False, True):
        s0, h1, s = torch.empty(N, C, device=DEV), torch.empty(N, csq, device=DEV), torch.empty(N, C, device=DEV)
        y = torch.empty_like(x)
        if fused:
            L.call('ewvit_se_forward', L.ptr(x), L.dt(x), N, HW, C, L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), csq,
                   L.ptr(s0), L.ptr(h1), L.ptr(s), L.ptr(y), L.ptr(ws), L.stream(x))
        else:
            L.call('ewvit_se_squeeze_mlp_fwd', L.ptr(x), L.dt(x), N, HW, C, L.ptr(w1), L.ptr(b1), L.ptr(w2),
                   L.ptr(b2), csq, L.ptr(s0), L.ptr(h1), L.ptr(s), L.ptr(ws), L.stream(x))
            L.call('ewvit_se_scale', L.ptr(x), L.dt(x), L.ptr(s), None, L.ptr(y), N, HW, C, L.stream(x))
        out.append((s0, h1, s, y))
    torch.cuda.synchronize()
    for a, b in zip(*out):
        assert torch.equal(a, b)
    ref = x.float() * out[0][2].view(N, 1, C)
    assert float((out[1][3].float() - ref).abs().max()) <= 2 ** -7 * float(ref.abs().max())


@pytest.mark.parametrize('N,C,H,csq', [(64, 1536, 7, 64), (64, 960, 14, 40), (3, 200, 5, 6)])
def test_bn_act_se_squeeze_matches_separate_passes(N, C, H, csq, monkeypatch):
    """bn_act_se with the depthwise conv's partial statistics: the fused BatchNorm apply + SE
    squeeze (ewvit_bn_act_se_squeeze + ewvit_se_gate_excite) gives the separate passes' bits —
    output, saved statistics, running statistics, counter — and the same gradients."""
    import ewvit
    import ewvit.se as ese
    g = torch.Generator().manual_seed(C + H)
    x = (torch.randn(N, C, H, H, generator=g) * 0.7 + 0.2).to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    wd = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).to(DEV)
    w1 = (torch.randn(csq, C, 1, 1, generator=g) / C ** 0.5).to(DEV)
    b1 = (torch.randn(csq, generator=g) * 0.1).to(DEV)
    w2 = (torch.randn(C, csq, 1, 1, generator=g) / csq ** 0.5).to(DEV)
    b2 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    dy = torch.randn(N, C, H, H, generator=g).to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    outs = []
    for fused in (False, True):
        monkeypatch.setattr(ese, '_BN_SQUEEZE', fused)
        bn = torch.nn.BatchNorm2d(C, eps=1e-3).train().to(DEV)
        xd = x.clone().requires_grad_(True)
        ps = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
        r = ewvit.ops.dwconv3x3_bn_stats(xd, wd, 1, bn.running_mean)
        assert r is not None
        y = ewvit.bn_act_se(r[0], bn, 'silu', *ps, partials=r[1:])
        y.backward(dy)
        torch.cuda.synchronize()
        outs.append((y.detach(), xd.grad, bn.running_mean.clone(), bn.running_var.clone(),
                     bn.num_batches_tracked.clone(), bn.weight.grad, [p.grad for p in ps]))
    a, b = outs
    for u, v in zip(a[:6], b[:6]):
        assert torch.equal(u, v)
    for u, v in zip(a[6], b[6]):
        assert torch.equal(u, v)


@pytest.mark.parametrize('N,C,H,W,csq,act', [(64, 1536, 7, 7, 64, 'silu'), (64, 960, 14, 14, 40, 'silu'),
                                             (5, 24, 9, 11, 6, 'relu'), (3, 200, 5, 3, 6, None)])
def test_bn_se_bwd_matches_two_pass_path(N, C, H, W, csq, act, monkeypatch):
    """ewvit_bn_se_bwd (the BatchNorm's backward sums split per frame and formed in the SE
    squeeze pass) against ewvit_se_squeeze_mlp_bwd + ewvit_bn_bwd_se (a reduction pass over the
    whole map): the same fp32 sums in another order — SE parameter gradients to 1e-5, dgamma /
    dbeta to 1e-4, dx to one bf16 rounding on < 5 % of its elements."""
    import ewvit
    import ewvit.se as ese
    g = torch.Generator().manual_seed(C + H)
    x = (torch.randn(N, C, H, W, generator=g) * 1.5 + 0.3).to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    w1 = (torch.randn(csq, C, 1, 1, generator=g) / C ** 0.5).to(DEV)
    b1 = (torch.randn(csq, generator=g) * 0.1).to(DEV)
    w2 = (torch.randn(C, csq, 1, 1, generator=g) / csq ** 0.5).to(DEV)
    b2 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    dy = torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    gam, bet = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.2
    outs = []
    for fused in (True, False):
        monkeypatch.setattr(ese, '_BN_SE_FUSED', fused)
        bn = torch.nn.BatchNorm2d(C, eps=1e-3).train().to(DEV)
        with torch.no_grad():
            bn.weight.copy_(gam)
            bn.bias.copy_(bet)
        xd = x.clone().requires_grad_(True)
        ps = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
        y = ewvit.bn_act_se(xd, bn, act, *ps)
        y.backward(dy)
        outs.append((y, xd.grad, bn.weight.grad, bn.bias.grad, [p.grad for p in ps]))
    a, b = outs
    assert torch.equal(a[0], b[0])
    for p, q in zip(a[4], b[4]):
        assert rel(p, q) < 1e-5          # ds summed in another order (fp32 reassociation only)
    assert rel(a[2], b[2]) < 1e-4 and rel(a[3], b[3]) < 1e-4
    d = (a[1].float() - b[1].float()).abs()
    assert float(d.max()) <= 2 ** -7 * float(b[1].float().abs().max())
    assert float((d > 0).float().mean()) < 0.05
