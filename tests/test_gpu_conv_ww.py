"""Wide-wave fwd / input-gradient blocks of the LDS-DMA conv (csrc/conv.hip
ewvit_conv2d_set_ww: each wave 64 x 128 of a 256 x 128 or 128 x 128 tile).  The grid
threshold is lowered so small shapes take them.  Each output element accumulates the same
K-tiles in the same order through the same MFMA as the 4-wave 64 x 64 blocks, so outputs and
input gradients must be BIT-identical to the default kernels (themselves checked against
torch fp32 in test_gpu_conv.py); the BatchNorm partial statistics change their row count
(256-row tiles) and must give the same batch statistics."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(params=[1, 2, 3], ids=['ww1', 'ww2', 'ww3'])
def ww(request):
    import ewvit
    lib = ewvit._lib.load()
    prev_min = lib.ewvit_conv2d_set_ww_min(0)
    prev = lib.ewvit_conv2d_set_ww(0)
    yield lib, request.param
    lib.ewvit_conv2d_set_ww(prev)
    lib.ewvit_conv2d_set_ww_min(prev_min)


def _run(lib, v, fn):
    prev = lib.ewvit_conv2d_set_ww(v)
    try:
        return fn()
    finally:
        lib.ewvit_conv2d_set_ww(prev)


@pytest.mark.parametrize('N,Cin,Cout,H,W,stride,k,levels', [
    (2, 64, 128, 28, 28, 1, 3, 1),
    (1, 128, 128, 16, 16, 1, 3, 3),      # level-major input (the multiscale conv)
    (3, 64, 384, 30, 31, 1, 3, 1),       # 3 column tiles, ragged M
    (2, 256, 128, 9, 13, 1, 1, 1),       # 1x1
    (2, 128, 128, 15, 13, 2, 3, 1),      # stride 2 forward (the dgrad takes the parity classes)
    (4, 128, 128, 56, 56, 1, 3, 1),
])
def test_ww_bit_identical(N, Cin, Cout, H, W, stride, k, levels, ww):
    import ewvit.conv as ec
    lib, v = ww
    g = torch.Generator().manual_seed(N * 31 + Cin + Cout + H)
    z = torch.randn(levels * N, Cin, H, W, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    w = (torch.randn(Cout, levels * Cin, k, k, generator=g) / (k * k * levels * Cin) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    dy = torch.randn(N, Cout, Ho, Wo, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)

    def step():
        zz = z.clone().requires_grad_(True)
        ww_ = w.clone().requires_grad_(True)
        y = ec.conv2d(zz, ww_, b, stride, levels)
        y.backward(dy)
        torch.cuda.synchronize()
        return y.detach().clone(), zz.grad.clone(), ww_.grad.clone()

    y0, dz0, dw0 = _run(lib, 0, step)
    y1, dz1, dw1 = _run(lib, v, step)
    assert torch.equal(y0, y1)
    assert torch.equal(dz0, dz1)
    assert torch.equal(dw0, dw1)          # the weight gradient does not take these blocks


@pytest.mark.parametrize('cin,cout,k,hw,groups', [(64, 128, 3, 32, 1), (128, 384, 3, 16, 1), (64, 128, 3, 32, 2)])
def test_ww_bn_partials(cin, cout, k, hw, groups, ww):
    """The forward's BatchNorm partial sums (256-row tiles for variants 1 / 3) reduce to the
    statistics of the stored output."""
    import ewvit
    import ewvit.conv as ec
    lib, v = ww
    torch.manual_seed(cin + cout + hw)
    x = (torch.randn(4, cin, hw, hw, device=DEV) * 1.5 + 0.3).to(torch.bfloat16).to(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, k, k, device=DEV) / (k * k * cin) ** 0.5
    shift = torch.linspace(-0.5, 0.5, cout, device=DEV)
    prev = lib.ewvit_conv2d_set_ww(v)
    try:
        rows = ec.bn_stat_rows(x, w, 1)
        assert rows == (128 if v == 2 else 256)
        out = ec.conv2d_bn_stats(x, w, None, 1, shift, groups=groups)
        assert out is not None
        y, part, shifts, nrc = out
        torch.cuda.synchronize()
    finally:
        lib.ewvit_conv2d_set_ww(prev)
    yf = y.float().permute(0, 2, 3, 1).reshape(groups, -1, cout).double()
    p = part.reshape(groups, nrc, 2 * cout).double().sum(1)
    sh = shifts.reshape(-1, cout).double()
    n = yf.shape[1]
    mean = p[:, :cout] / n + sh
    var = p[:, cout:] / n - (p[:, :cout] / n) ** 2
    assert torch.allclose(mean, yf.mean(1), atol=1e-4, rtol=1e-4)
    assert torch.allclose(var, yf.var(1, unbiased=False), atol=1e-4, rtol=1e-3)
