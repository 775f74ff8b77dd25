"""Fused BatchNorm2d + activation kernels (csrc/batchnorm.hip) through the C-ABI,
vs torch fp32 F.batch_norm + activation on the same (bf16-rounded) input.

Tolerance: bf16 output = one rounding of an fp32 result: 2^-7 of scale (plus
exp/rsqrt ulps); fp32 output 1e-4; gradients 2e-3 of scale (fp32 reductions in a
different order); running statistics 1e-4.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


def ref_bn(x, w, b, rm, rv, training, act, groups):
    """torch reference: `groups` sequential F.batch_norm calls on batch slices."""
    outs = []
    n = x.shape[0] // groups
    for g in range(groups):
        y = torch.nn.functional.batch_norm(x[g * n:(g + 1) * n], rm, rv, w, b, training, 0.1, 1e-3)
        outs.append(torch.relu(y) if act == 'relu' else torch.nn.functional.silu(y) if act == 'silu' else y)
    return torch.cat(outs)


@pytest.mark.parametrize('shape,groups', [((64, 960, 14, 14), 1), ((6, 56, 20, 20), 3), ((4, 24, 33, 33), 1),
                                          ((8, 1280, 7, 7), 1), ((64, 128), 1), ((6, 128, 12, 12), 2),
                                          ((48, 64, 56, 56), 3), ((64, 1536, 7, 7), 1), ((2, 2048, 3, 3), 1)])
@pytest.mark.parametrize('act', [None, 'relu', 'silu'])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_bn_act_train(shape, groups, act, dtype):
    import ewvit
    g = torch.Generator().manual_seed(shape[1] + groups)
    x = (torch.randn(shape, generator=g) * 2 + 0.5).to(dtype)
    C = shape[1]
    w = torch.randn(C, generator=g) * 0.5 + 1
    b = torch.randn(C, generator=g) * 0.1
    rm0, rv0 = torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5
    xr = x.float().clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rm_r, rv_r = rm0.clone(), rv0.clone()
    yr = ref_bn(xr, wr, br, rm_r, rv_r, True, act, groups)
    dy = torch.randn(yr.shape, generator=g).to(dtype)
    yr.backward(dy.float())
    xd = x.to(DEV)
    if xd.dim() == 4:
        xd = xd.to(memory_format=torch.channels_last)
    xd.requires_grad_(True)
    wd, bd = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    rm_d, rv_d = rm0.to(DEV), rv0.to(DEV)
    counter = torch.full((), 7, dtype=torch.int64, device=DEV)
    y = ewvit.batch_norm_act_params(xd, wd, bd, rm_d, rv_d, True, 0.1, 1e-3, act, groups, counter)
    y.backward(dy.to(DEV))
    assert int(counter) == 7 + groups
    tol = 2 ** -7 if dtype == torch.bfloat16 else 1e-4
    assert y.dtype == dtype
    assert rel(y.float(), yr) < tol
    assert rel(rm_d, rm_r) < 1e-4 and rel(rv_d, rv_r) < 1e-4
    # ReLU: where the reference pre-activation is within rounding of 0 the two
    # implementations may take different sides of the kink (dx = 0 vs dy*k);
    # compare dx away from it
    keep = torch.ones_like(yr, dtype=torch.bool)
    if act == 'relu':
        with torch.no_grad():
            z = ref_bn(x.float(), w, b, rm0.clone(), rv0.clone(), True, None, groups)
        keep = z.abs() > 1e-5 * float(z.abs().max())
    assert rel(xd.grad.float().cpu()[keep], xr.grad[keep]) < (2e-2 if dtype == torch.bfloat16 else 2e-3)
    assert rel(wd.grad, wr.grad) < 2e-3
    assert rel(bd.grad, br.grad) < 2e-3


@pytest.mark.parametrize('act', [None, 'relu', 'silu'])
def test_bn_act_eval(act):
    import ewvit
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 64, 9, 9, generator=g)
    w, b = torch.randn(64, generator=g), torch.randn(64, generator=g)
    rm, rv = torch.randn(64, generator=g), torch.rand(64, generator=g) + 0.5
    yr = ref_bn(x, w, b, rm.clone(), rv.clone(), False, act, 1)
    y = ewvit.batch_norm_act_params(x.to(DEV).to(memory_format=torch.channels_last), w.to(DEV), b.to(DEV),
                                    rm.to(DEV), rv.to(DEV), False, 0.1, 1e-3, act)
    assert rel(y, yr) < 1e-5


def test_bn_stats_stable_with_large_mean():
    """Sums shifted by a sample of each channel: a large common offset must not destroy the variance."""
    import ewvit
    x = torch.randn(16, 64, 32, 32) * 0.01 + 300.0
    rm, rv = torch.zeros(64), torch.ones(64)
    yr = ref_bn(x.double(), None, None, rm.double(), rv.double(), True, None, 1)
    rmd, rvd = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    y = ewvit.batch_norm_act_params(x.to(DEV).to(memory_format=torch.channels_last), None, None, rmd, rvd, True,
                                    0.1, 1e-3, None)
    assert rel(y, yr) < 5e-3


@pytest.mark.parametrize('cin,cout,k,stride,hw', [(256, 512, 1, 1, 7), (64, 256, 1, 1, 14), (128, 160, 3, 2, 13),
                                                 (64, 64, 3, 1, 9)])
def test_conv_bn_stats_in_epilogue(cin, cout, k, stride, hw):
    """ConvBNAct training forward with the BatchNorm batch statistics summed in the
    conv's epilogue (ewvit_conv2d_fwd_bn + ewvit_bn_fwd_partials) matches the unfused
    conv -> BN(+SiLU) path: output, running stats, counter, and all gradients."""
    import ewvit
    from network.efficientnet import ConvBNAct
    torch.manual_seed(cin + cout + k)
    m1 = ConvBNAct(cin, cout, k, stride).to(DEV)
    m2 = ConvBNAct(cin, cout, k, stride).to(DEV)
    m2.load_state_dict(m1.state_dict())
    with torch.no_grad():
        for m in (m1, m2):
            m[1].running_mean.copy_(torch.linspace(-0.5, 0.5, cout))   # shift used by the fused sums
    x = (torch.randn(6, cin, hw, hw) * 1.5 + 0.3).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    assert ewvit.conv.bn_stat_rows(x, m1[0].weight, stride) > 0
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    y1 = m1(x1)                                   # fused statistics path
    y2 = ewvit.batch_norm_act(m2[0](x2), m2[1], 'silu')   # conv, then the full BN
    dy = torch.randn(y1.shape, device=DEV).to(torch.bfloat16)
    y1.backward(dy)
    y2.backward(dy)
    assert rel(y1.float(), y2.float()) < 2 ** -7
    assert rel(m1[1].running_mean, m2[1].running_mean) < 1e-4
    assert rel(m1[1].running_var, m2[1].running_var) < 1e-4
    assert int(m1[1].num_batches_tracked) == int(m2[1].num_batches_tracked) == 1
    assert rel(x1.grad.float(), x2.grad.float()) < 2e-2
    assert rel(m1[0].weight.grad, m2[0].weight.grad) < 1e-2
    assert rel(m1[1].weight.grad, m2[1].weight.grad) < 1e-2
    assert rel(m1[1].bias.grad, m2[1].bias.grad) < 1e-2


@pytest.mark.parametrize('hw', [64, 40])
def test_mwt_epilogue_stats_match_plain(hw, monkeypatch):
    """MWT forward/backward with the BN statistics of its convs summed in the conv
    epilogues (per-level groups for the fusion conv, folded partial rows) equals the
    plain conv -> BN path: outputs, running stats and parameter gradients."""
    import network.mwt as mw
    torch.manual_seed(3)
    m1 = mw.MWT(3, 128, 3).to(DEV).to(memory_format=torch.channels_last)
    m2 = mw.MWT(3, 128, 3).to(DEV).to(memory_format=torch.channels_last)
    m2.load_state_dict(m1.state_dict())
    x = torch.randn(2, 3, hw, hw, device=DEV)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y1 = m1(x)
    calls = []
    real = mw._epi_stats
    monkeypatch.setattr(mw, '_epi_stats', lambda *a, **k: calls.append(1))
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y2 = m2(x)
    monkeypatch.setattr(mw, '_epi_stats', real)
    assert len(calls) >= 3
    g = torch.randn(y1.shape, device=DEV)
    y1.float().mul(g).sum().backward()
    y2.float().mul(g).sum().backward()
    assert rel(y1.float(), y2.float()) < 2e-2
    for (n, b1), b2 in zip(m1.named_buffers(), m2.buffers()):
        if b1.dtype.is_floating_point:
            assert rel(b1, b2) < 1e-3, n
        else:
            assert torch.equal(b1, b2), n
    # gradients pass the freq_pool max-pool, whose bf16 near-ties may route a pixel's
    # gradient differently once the statistics' summation order changes: compare by
    # direction, not elementwise
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        # a conv bias in front of a BatchNorm has an exactly-zero true gradient: its
        # computed value is rounding noise, not compared
        if p1.grad is not None and not (n.endswith('0.bias') or n.endswith('1.bias') and 'freq_pool' in n):
            cos = torch.nn.functional.cosine_similarity(p1.grad.flatten().double(), p2.grad.flatten().double(), 0)
            assert float(cos) > 0.995, (n, float(cos))
