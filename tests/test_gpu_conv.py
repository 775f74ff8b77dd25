"""Implicit-GEMM 3x3 conv kernels (csrc/conv.hip) through the C-ABI, vs torch
fp32 conv2d on the same bf16-rounded operands.

Tolerance: outputs / input-grads are rounded to bf16 once (fp32 accumulation of
bf16 products, so only summation order and the final rounding differ):
max |err| <= 2^-7 of scale; weight/bias grads (fp32 out) <= 1e-3 of scale.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


@pytest.mark.parametrize('N,Cx,Cin,Cout,H,W,stride', [
    (2, 64, 64, 128, 28, 28, 1),
    (1, 384, 384, 128, 16, 16, 1),
    (2, 128, 128, 128, 15, 13, 2),
    (3, 64, 54, 128, 20, 20, 1),      # fusion: 54 real channels zero-padded to 64
    (2, 32, 32, 64, 9, 9, 2),
    (1, 8, 8, 8, 5, 7, 1),
])
def test_conv3x3_fwd_bwd(N, Cx, Cin, Cout, H, W, stride):
    import ewvit.conv as ec
    g = torch.Generator().manual_seed(Cx * 7 + H)
    x = torch.randn(N, Cx, H, W, generator=g).to(torch.bfloat16)
    if Cx > Cin:
        x[:, Cin:] = 0
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5)
    b = torch.randn(Cout, generator=g)
    xr = x[:, :Cin].float().clone().requires_grad_(True)
    wr = w.to(torch.bfloat16).float().clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, br, stride=stride, padding=1)
    dy = torch.randn(yr.shape, generator=g).to(torch.bfloat16)
    yr.backward(dy.float())
    xd = x.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    wd, bd = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    y = ec.conv3x3(xd, wd, bd, stride)
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
