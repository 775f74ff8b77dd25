"""The 1x1 stride-1 weight-gradient kernel (csrc/conv.hip conv_wgrad_1x1_kernel) through the
C-ABI, on the backbone's 1x1 shapes (MBConv expand / project of stages 2-6 and the head conv of
sfe.py:111-113's EfficientNetV2-S at 224^2, 64 frames) plus ragged tiles:
  * against torch fp32 of the same bf16 operands, dW = dy^T x (1e-5 of the largest entry);
  * against the generic LDS-DMA kernel (ewvit_conv2d_set_wgrad_1x1(0, ...)): same fp32 products,
    other split boundaries, so equal to summation order (1e-6);
  * one split writes dW directly; accumulate = 1 adds into dW; a parameter-strided dW
    (channels-last weight) goes through the reduce pass."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _wgrad(lib, L, x, dy, dw, ws, N, H, W, Cin, Cout, acc=0):
    L.call('ewvit_conv2d_bwd_weight', L.ptr(x), L.ptr(dy), L.ptr(dw), None, acc, N, H, W, Cin, Cout, 1, 1, 0, 0,
           Cin, dw.stride(0), dw.stride(1), dw.stride(3), L.ptr(ws), L.stream(dw))


@pytest.mark.parametrize('N,Cin,H,W,Cout', [
    (64, 256, 7, 7, 1536),     # stage 6 expand
    (64, 1536, 7, 7, 256),     # stage 6 project
    (64, 160, 14, 14, 960),    # stage 5 expand: ragged ci tile (160 = 128 + 32)
    (64, 960, 14, 14, 160),    # stage 5 project: ragged co tile
    (64, 128, 14, 14, 512),    # stage 4 expand
    (64, 192, 56, 56, 48),     # stage 2 project: 48-channel co tile, 200704 pixels
    (64, 256, 7, 7, 1280),     # head conv
    (3, 96, 13, 11, 200),      # ragged everything, 429 pixels (one split: dW written directly)
])
def test_wgrad_1x1(N, Cin, H, W, Cout):
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    lib = L.load()
    g = torch.Generator().manual_seed(Cin * 7 + Cout + H)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, Cout, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ws = torch.empty(int(lib.ewvit_conv2d_bwd_weight_workspace(N, H, W, Cin, Cout, 1, 1)) // 4 + 64, device=DEV)
    dw = torch.full((Cout, Cin, 1, 1), float('nan'), device=DEV)
    _wgrad(lib, L, x, dy, dw, ws, N, H, W, Cin, Cout)
    base = torch.full((Cout, Cin, 1, 1), 0.25, device=DEV)
    dwa = base.clone()
    _wgrad(lib, L, x, dy, dwa, ws, N, H, W, Cin, Cout, acc=1)
    # a dW with the parameter's channels-last strides (s_ci = 1 still, s_co = Cin): and a
    # transposed view (s_ci = Cout) that cannot take the direct store
    dwt = torch.full((Cin, Cout, 1, 1), float('nan'), device=DEV).permute(1, 0, 2, 3)
    _wgrad(lib, L, x, dy, dwt, ws, N, H, W, Cin, Cout)
    # the shipped knobs (conv.hip g_w1_*) are what the kernel above ran with, on every shape
    assert [lib.ewvit_conv2d_wgrad_1x1_config(i) for i in range(3)] == [256, 8, 2]
    prev = lib.ewvit_conv2d_set_wgrad_1x1(0, 0, 0)       # generic kernel; the other knobs kept
    try:
        ws2 = torch.empty(int(lib.ewvit_conv2d_bwd_weight_workspace(N, H, W, Cin, Cout, 1, 1)) // 4 + 64, device=DEV)
        dw_gen = torch.empty((Cout, Cin, 1, 1), device=DEV)
        _wgrad(lib, L, x, dy, dw_gen, ws2, N, H, W, Cin, Cout)
        torch.cuda.synchronize()
    finally:
        lib.ewvit_conv2d_set_wgrad_1x1(prev, 0, 0)
    assert [lib.ewvit_conv2d_wgrad_1x1_config(i) for i in range(3)] == [256, 8, 2]
    ref = dy.double().permute(1, 0, 2, 3).reshape(Cout, -1) @ x.double().permute(0, 2, 3, 1).reshape(-1, Cin)
    ref = ref.float().reshape(Cout, Cin, 1, 1)
    scale = float(ref.abs().max())
    assert not torch.isnan(dw).any()
    err = float((dw - ref).abs().max()) / scale
    assert err < 1e-5, err
    assert float((dw_gen - dw).abs().max()) / scale < 1e-6
    assert float((dwa - base - dw).abs().max()) / scale < 1e-6
    assert torch.equal(dwt, dw)
