"""Implicit-GEMM conv kernels (csrc/conv.hip, kernel 1x1 / 3x3) through the C-ABI,
vs torch fp32 conv2d on the same bf16-rounded operands.

Tolerance: outputs / input-grads are rounded to bf16 once (fp32 accumulation of
bf16 products, so only summation order and the final rounding differ):
max |err| <= 2^-7 of scale; weight/bias grads (fp32 out) <= 1e-3 of scale.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(params=[1, 0, 'wide', 'narrow'], ids=['glds', 'regstage', 'glds-wgrad-wide', 'glds-wgrad-narrow'])
def glds(request):
    """Run each case on the LDS-DMA kernels (weight gradient: auto tile width, always the
    256-column tiles where the shape allows them, never) and on the register-staged kernels
    (the fallback of the shapes the LDS-DMA kernels refuse)."""
    import ewvit
    lib = ewvit._lib.load()
    p = request.param
    v, w = (1, {'wide': 2, 'narrow': 0}[p]) if isinstance(p, str) else (p, 4)
    prev = lib.ewvit_conv2d_set_glds(v)
    prevw = lib.ewvit_conv2d_set_wgrad_wide(w)
    yield v
    lib.ewvit_conv2d_set_glds(prev)
    lib.ewvit_conv2d_set_wgrad_wide(prevw)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


@pytest.mark.parametrize('N,Cx,Cin,Cout,H,W,stride,k', [
    (2, 64, 64, 128, 28, 28, 1, 3),
    (1, 384, 384, 128, 16, 16, 1, 3),
    (2, 128, 128, 128, 15, 13, 2, 3),
    (3, 64, 54, 128, 20, 20, 1, 3),      # fusion: 54 real channels zero-padded to 64
    (2, 56, 54, 64, 12, 12, 1, 3),       # 56-channel input: K-tiles straddle taps
    (2, 32, 32, 64, 9, 9, 2, 3),
    (1, 8, 8, 8, 5, 7, 1, 3),
    (2, 24, 24, 96, 17, 17, 2, 3),       # backbone FusedMBConv expand, stride 2
    (2, 96, 96, 48, 14, 14, 1, 1),       # backbone 1x1 project
    (2, 64, 64, 256, 7, 9, 1, 1),        # 1x1 expand
    (1, 256, 256, 1280, 7, 7, 1, 1),     # head 1x1
    (2, 48, 48, 24, 10, 11, 2, 1),       # 1x1 stride 2, K-tile straddles nothing
    (4, 128, 128, 128, 56, 56, 1, 3),    # many M tiles, split pixel reduction
    (3, 64, 64, 384, 30, 31, 1, 3),      # 3 N tiles, ragged M
    (2, 128, 128, 128, 57, 55, 2, 3),    # odd sizes, stride 2
    (5, 64, 64, 64, 33, 35, 1, 1),       # 1x1, 64-wide output tile
    (4, 1536, 1536, 256, 7, 7, 1, 1),    # 1x1 project: long K, few tiles
    (3, 256, 256, 1536, 7, 7, 1, 1),     # 1x1 expand: long-K dgrad
    (2, 192, 192, 160, 9, 9, 1, 3),      # 3x3, few tiles, 27 K-tiles
    (2, 160, 160, 64, 9, 9, 1, 1),       # Cin 160: LDS-DMA fwd with K padded to 192 per tap
    (2, 160, 160, 48, 11, 10, 2, 3),     # the same, 3x3 stride 2
    (2, 960, 960, 160, 7, 7, 1, 1),      # 1x1 project: dgrad K = 160 per tap (ragged last K-tile)
    (2, 192, 192, 48, 14, 14, 1, 1),     # dgrad K = 48: one ragged K-tile
    (2, 48, 48, 192, 15, 14, 1, 3),      # 3x3 fwd Cin 48: ragged K-tile in every tap
    (1, 16, 16, 64, 20, 19, 1, 3),       # Cin 16 (the MWT seperate conv's input)
    (2, 24, 24, 96, 24, 24, 2, 3),       # stage-2 entry: parity-class dgrad into 24 channels (32-wide tiles)
    (1, 32, 32, 64, 18, 18, 2, 3),       # dgrad into exactly 32 channels
    (2, 24, 24, 24, 21, 19, 1, 3),       # stage 1 (24 -> 24): small-channel direct conv fwd + dgrad
    (1, 24, 24, 24, 112, 112, 1, 3),     # the same at 112^2 (TH-row bands, full-width LDS tiles)
    (2, 16, 16, 16, 9, 13, 1, 3),        # Cin / Cout 16: both directions on the small-channel kernel
    (1, 24, 24, 8, 7, 5, 1, 3),          # one 16-wide output tile, rows < the band height
    (2, 16, 16, 64, 10, 16, 1, 3),       # small-channel wgrad (W % 8 == 0): 16 -> 64 with bias
    (3, 24, 24, 24, 7, 24, 1, 3),        # small-channel wgrad, odd H (a 1-row tail band)
    (64, 160, 160, 960, 14, 14, 1, 1),   # bench-size stage-5 expand: many pixel splits
    (64, 256, 256, 1536, 7, 7, 1, 1),    # bench-size stage-6 expand
])
def test_conv_fwd_bwd(N, Cx, Cin, Cout, H, W, stride, k, glds):
    import ewvit.conv as ec
    g = torch.Generator().manual_seed(Cx * 7 + H + k)
    x = torch.randn(N, Cx, H, W, generator=g).to(torch.bfloat16)
    if Cx > Cin:
        x[:, Cin:] = 0
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (k * k * Cin) ** 0.5)
    b = torch.randn(Cout, generator=g)
    xr = x[:, :Cin].float().clone().requires_grad_(True)
    wr = w.to(torch.bfloat16).float().clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, br, stride=stride, padding=k // 2)
    dy = torch.randn(yr.shape, generator=g).to(torch.bfloat16)
    yr.backward(dy.float())
    xd = x.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    wd, bd = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    y = ec.conv2d(xd, wd, bd, stride)
    assert y.shape == yr.shape and y.dtype == torch.bfloat16
    assert y.is_contiguous(memory_format=torch.channels_last)
    y.backward(dy.to(DEV))
    assert rel(y, yr) < 2 ** -7
    assert rel(xd.grad[:, :Cin], xr.grad) < 2 ** -7
    if Cx > Cin:
        assert float(xd.grad[:, Cin:].abs().max()) == 0.0
    # weight grads: the kernel sees bf16 x (as torch does above) and bf16 dy
    assert rel(wd.grad, wr.grad) < 1e-3
    assert rel(bd.grad, br.grad) < 1e-3


@pytest.mark.parametrize('levels,N,C,Cout,H,W', [(3, 2, 128, 128, 14, 14), (2, 3, 32, 64, 9, 10),
                                               (3, 4, 128, 128, 40, 41)])
def test_conv_level_major_input(levels, N, C, Cout, H, W, glds):
    """levels > 1: the conv reads z [L*N, C, H, W] as cat(z.chunk(L), 1) in place
    (the multiscale fusion input, mwt.py:112) and returns dz in z's layout."""
    import ewvit.conv as ec
    g = torch.Generator().manual_seed(levels * 100 + C)
    z = torch.randn(levels * N, C, H, W, generator=g).to(torch.bfloat16)
    w = torch.randn(Cout, levels * C, 3, 3, generator=g) / (9 * levels * C) ** 0.5
    b = torch.randn(Cout, generator=g)
    zr = z.float().clone().requires_grad_(True)
    wr = w.to(torch.bfloat16).float().clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(torch.cat(zr.chunk(levels), 1), wr, b, padding=1)
    dy = torch.randn(yr.shape, generator=g).to(torch.bfloat16)
    yr.backward(dy.float())
    zd = z.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = ec.conv2d(zd, wd, b.to(DEV), 1, levels)
    y.backward(dy.to(DEV))
    assert y.shape == yr.shape
    assert rel(y, yr) < 2 ** -7
    assert zd.grad.shape == z.shape and rel(zd.grad, zr.grad) < 2 ** -7
    assert rel(wd.grad, wr.grad) < 1e-3


@pytest.mark.parametrize('Cx,Cin,k', [(64, 64, 3), (64, 54, 3), (96, 96, 1), (64, 60, 1)])
def test_conv_weight_grad_in_param_layout(Cx, Cin, k):
    """dW is written straight into the parameter's memory format (channels-last conv
    weights, as the model holds them) and only for the real input channels."""
    import ewvit.conv as ec
    g = torch.Generator().manual_seed(Cx + Cin + k)
    x = torch.randn(3, Cx, 13, 11, generator=g).to(torch.bfloat16)
    x[:, Cin:] = 0
    w = torch.randn(48, Cin, k, k, generator=g) / (k * k * Cin) ** 0.5
    xr = x[:, :Cin].float().clone().requires_grad_(True)
    wr = w.to(torch.bfloat16).float().clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, padding=k // 2)
    dy = torch.randn(yr.shape, generator=g).to(torch.bfloat16)
    yr.backward(dy.float())
    xd = x.to(DEV).to(memory_format=torch.channels_last)
    wd = w.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    y = ec.conv2d(xd, wd, None, 1)
    y.backward(dy.to(DEV))
    assert wd.grad.stride() == wd.stride()
    assert rel(wd.grad, wr.grad) < 1e-3


def test_step_wide_weight_packing():
    """conv.packed(): every registered weight packed by one multi-tensor launch; the
    convs inside read those packs (bitwise the per-call packs), and a weight updated
    between steps is re-packed at the next scope entry."""
    import ewvit.conv as ec
    g = torch.Generator().manual_seed(11)
    shapes = [(64, 64, 3), (128, 54, 3), (256, 1536, 1), (40, 24, 1)]
    ws = [(torch.randn(co, ci, k, k, generator=g) * 0.1).to(DEV).requires_grad_(True) for co, ci, k in shapes]
    ws[1].data = ws[1].data.contiguous(memory_format=torch.channels_last)
    xs = [torch.randn(2, (ci + 7) // 8 * 8 if ci % 8 else ci, 9, 9, generator=g).to(torch.bfloat16).to(DEV)
          .contiguous(memory_format=torch.channels_last).requires_grad_(True) for _, ci, _ in shapes]
    for x, (_, ci, _) in zip(xs, shapes):
        with torch.no_grad():
            x[:, ci:] = 0

    def run():
        outs = []
        for x, w in zip(xs, ws):
            y = ec.conv2d(x, w, None, 1)
            y.float().square().sum().backward()
            outs.append((y.detach().clone(), x.grad.clone(), w.grad.clone()))
            x.grad = None
            w.grad = None
        return outs
    ref = run()                        # per-call packs; registers the weights
    with ec.packed():
        assert all(ec._cached_pack(w, x.shape[1], True) is not None for x, w in zip(xs, ws))
        got = run()
    for a, b in zip(ref, got):
        for u, v in zip(a, b):
            assert torch.equal(u, v)
    with torch.no_grad():
        for w in ws:
            w.mul_(-0.5)
    ref2 = run()
    with ec.packed():
        got2 = run()
    for a, b in zip(ref2, got2):
        for u, v in zip(a, b):
            assert torch.equal(u, v)
    assert not torch.equal(ref[0][0], ref2[0][0])


def test_conv_big_narrow_dgrad_256_row_blocks():
    """A <= 64-column input gradient over > 4096 row tiles takes 256-row blocks (the MWT fusion
    conv's 56-channel dgrad over 2.4 M pixels): against torch's fp32 conv on the GPU for the same
    bf16-rounded operands."""
    import ewvit.conv as ec
    g = torch.Generator().manual_seed(56)
    N, Cin, Cout, H = 44, 56, 128, 112            # 551,936 pixels = 4312 row tiles
    x = torch.randn(N, Cin, H, H, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5).to(DEV)
    dy = torch.randn(N, Cout, H, H, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    xd = x.clone().requires_grad_(True)
    ec.conv2d(xd, w, None, 1).backward(dy)
    xr = x.float().requires_grad_(True)
    torch.nn.functional.conv2d(xr, w.to(torch.bfloat16).float(), None, padding=1).backward(dy.float())
    assert rel(xd.grad, xr.grad) < 2 ** -7
