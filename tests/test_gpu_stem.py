"""The backbone stem's direct conv (csrc/stem.hip, ewvit_conv2d_stem_fwd): the frozen
features.0.0 Conv2d(3, 24, 3, stride 2) of EfficientNetV2-S (reference sfe.py:111-119
freezes backbone parameters 0-5), forward only, reading the fp32 NCHW frames.

Operands stay fp32 (the autocast reference rounds them to bf16 — the stem is the more
precise of the two at the same cost): against torch fp64 conv2d only the fp32 summation
order and the final bf16 rounding differ — max |err| <= 2^-8 of scale.  The BatchNorm partial sums it leaves are checked
against the sums of its own bf16 output (fp32 summation order only: 1e-5 relative), and
ConvBNAct on the stem path against fp64 conv / BatchNorm / SiLU."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


@pytest.mark.parametrize('N,Cin,Cout,H,W,stride,cl,bias,xdt', [
    (4, 3, 24, 224, 224, 2, True, False, torch.float32),     # the bench's stem
    (3, 3, 24, 37, 41, 2, False, True, torch.float32),       # odd sizes, contiguous weight
    (2, 1, 8, 19, 16, 1, True, True, torch.float32),
    (2, 4, 32, 33, 30, 2, False, False, torch.bfloat16),
    (1, 2, 16, 17, 17, 1, True, False, torch.bfloat16),
])
def test_stem_conv_vs_torch(N, Cin, Cout, H, W, stride, cl, bias, xdt):
    import ewvit
    g = torch.Generator().manual_seed(N * 100 + Cin * 10 + Cout + H)
    x = (torch.randn(N, Cin, H, W, generator=g) * 2).to(xdt)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / 5.0
    b = torch.randn(Cout, generator=g) if bias else None
    ref = torch.nn.functional.conv2d(x.double(), w.double(), None if b is None else b.double(), stride=stride, padding=1)
    wd = w.to(DEV)
    if cl:
        wd = wd.contiguous(memory_format=torch.channels_last)
    shift = torch.randn(Cout, generator=g) * 0.1
    y, part, shifts, nrc = ewvit.conv.stem_conv2d(x.to(DEV), wd, None if b is None else b.to(DEV), stride,
                                                  shift.to(DEV), stats=True)
    torch.cuda.synchronize()
    assert y.shape == ref.shape and y.dtype == torch.bfloat16
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert rel(y, ref) <= 2 ** -8
    # partial statistics: sums of (y - K) and (y - K)^2 over all pixels, K = shift
    d = y.float().permute(0, 2, 3, 1).reshape(-1, Cout).double().cpu() - shift.double()
    S, Q = part.reshape(-1, 2 * Cout)[:nrc].double().cpu().sum(0).split(Cout)
    assert nrc <= 256
    assert torch.equal(shifts.reshape(-1).cpu(), shift)
    assert rel(S, d.sum(0)) <= 1e-5 and rel(Q, (d * d).sum(0)) <= 1e-5
    # no statistics requested: the same output
    y2 = ewvit.conv.stem_conv2d(x.to(DEV), wd, None if b is None else b.to(DEV), stride)
    assert torch.equal(y2, y)


def test_stem_convbnact_vs_fp64():
    """ConvBNAct(3, 24, 3, 2) frozen, training under autocast: the ewvit stem (conv +
    epilogue sums + BN apply) against fp64 conv / BatchNorm / SiLU on the bf16-rounded
    conv output: output, running stats, counter; eval mode
    too; and the stem path must be the one that ran.  (The library conv it replaces —
    MIOpen's bf16 conv — measured a 2x larger elementwise error and a 0.6 % low batch
    variance on these inputs, tools/stem_diag.py, so it is not the yardstick.)"""
    import ewvit
    from network.efficientnet import ConvBNAct
    torch.manual_seed(3)
    m = ConvBNAct(3, 24, 3, 2).to(DEV).to(memory_format=torch.channels_last)
    for p in m.parameters():
        p.requires_grad_(False)
    with torch.no_grad():
        m[1].weight.uniform_(0.5, 1.5)
        m[1].bias.uniform_(-0.3, 0.3)
        m[1].running_mean.copy_(torch.linspace(-0.2, 0.2, 24))
    rm0, rv0 = m[1].running_mean.double().cpu(), m[1].running_var.double().cpu()
    x = torch.randn(8, 3, 64, 64, device=DEV)
    calls = []
    real = ewvit.conv.stem_conv2d

    def spy(*a, **k):
        calls.append(1)
        return real(*a, **k)
    ewvit.conv.stem_conv2d = spy
    try:
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y1 = m(x)
    finally:
        ewvit.conv.stem_conv2d = real
    assert calls == [1]
    xc, wc = x.double().cpu(), m[0].weight.double().cpu()
    c = torch.nn.functional.conv2d(xc, wc, stride=2, padding=1).to(torch.bfloat16).double()
    mean, var = c.mean(dim=(0, 2, 3)), c.var(dim=(0, 2, 3), unbiased=False)
    n = c.numel() // 24
    g, b = m[1].weight.double().cpu(), m[1].bias.double().cpu()

    def bn_silu(mu, v):
        z = (c - mu.view(1, -1, 1, 1)) / torch.sqrt(v.view(1, -1, 1, 1) + 1e-3) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)
        return z * torch.sigmoid(z)
    assert rel(y1.float(), bn_silu(mean, var)) <= 2 ** -7
    assert rel(m[1].running_mean, 0.9 * rm0 + 0.1 * mean) <= 1e-5
    assert rel(m[1].running_var, 0.9 * rv0 + 0.1 * var * n / (n - 1)) <= 1e-5
    assert int(m[1].num_batches_tracked) == 1
    m.eval()
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
        e = m(x)
    assert rel(e.float(), bn_silu(m[1].running_mean.double().cpu(), m[1].running_var.double().cpu())) <= 2 ** -7


def test_stem_needs_frozen_weights():
    """A stem whose weight takes a gradient is not the stem kernel's case (forward only):
    ConvBNAct keeps the library conv and the gradient flows."""
    import ewvit
    from network.efficientnet import ConvBNAct
    m = ConvBNAct(3, 24, 3, 2).to(DEV)
    x = torch.randn(2, 3, 32, 32, device=DEV)
    assert not ewvit.conv.stem_ok(x, m[0].weight, m[0].bias, 2)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = m(x)
    y.float().sum().backward()
    assert m[0].weight.grad is not None and float(m[0].weight.grad.abs().sum()) > 0
    with torch.no_grad():
        assert ewvit.conv.stem_ok(x, m[0].weight, m[0].bias, 2)
