"""3x3 convolution (pad 1, stride 1|2, bias) on the ewvit implicit-GEMM kernels
(csrc/conv.hip) — the MWT conv stack of network/mwt.py:23-72.

Activations are channels-last bf16 (the MFMA operand type); weights stay fp32
master parameters and are packed to bf16 [Cout][9][Cin] each call.  An input
may carry zero-padded channels (Cin_x > weight.shape[1]): the pack fills those
weight rows with zeros, so they contribute exactly nothing and receive no
gradient.
"""
import torch

from . import _lib as L



def _pack(weight, cin_pad, transposed):
    Cout, Cin = weight.shape[0], weight.shape[1]
    w = weight.detach().float().contiguous()
    shape = (Cout, 9, cin_pad) if not transposed else (cin_pad, 9, Cout)
    wp = torch.empty(shape, dtype=torch.bfloat16, device=weight.device)
    L.call('ewvit_conv3x3_pack_weight', L.ptr(w), L.ptr(wp), Cout, Cin, cin_pad, int(transposed), L.stream(wp))
    return wp


class Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride):
        L.require_gpu(x, weight)
        N, Cx, H, W = x.shape
        Cout, Cin = weight.shape[0], weight.shape[1]
        if Cx < Cin or weight.shape[2:] != (3, 3):
            raise ValueError(f'conv3x3: input has {Cx} channels, weight {tuple(weight.shape)}')
        xc = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wp = _pack(weight, Cx, False)
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        b = bias.detach().float().contiguous() if bias is not None else None
        work = {'flops': 2.0 * N * Ho * Wo * Cout * 9 * Cx, 'bytes': (xc.numel() + y.numel() + wp.numel()) * 2}
        L.call('ewvit_conv3x3_fwd', L.ptr(xc), L.ptr(wp), L.ptr(b), L.ptr(y), N, H, W, Cx, Cout, stride,
               L.stream(y), work=work)
        ctx.save_for_backward(xc, weight)
        ctx.cfg = (stride, bias is not None, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, weight = ctx.saved_tensors
        stride, has_bias, xdt = ctx.cfg
        N, Cx, H, W = xc.shape
        Cout, Cin = weight.shape[0], weight.shape[1]
        Ho, Wo = dy.shape[2], dy.shape[3]
        dyc = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wpt = _pack(weight, Cx, True)
            dx = torch.empty_like(xc, memory_format=torch.channels_last)
            work = {'flops': 2.0 * N * H * W * Cx * 9 * Cout, 'bytes': (dyc.numel() + dx.numel() + wpt.numel()) * 2}
            L.call('ewvit_conv3x3_bwd_data', L.ptr(dyc), L.ptr(wpt), L.ptr(dx), N, H, W, Cx, Cout, stride,
                   L.stream(dx), work=work)
            if xdt != torch.bfloat16:
                dx = dx.to(xdt)
        want_b = has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            wsb = L.load().ewvit_conv3x3_bwd_weight_workspace(N, H, W, Cx, Cout, stride)
            ws = torch.empty(wsb // 4, dtype=torch.float32, device=xc.device)
            dwf = torch.empty((Cout, Cx, 3, 3), dtype=torch.float32, device=xc.device)
            dbf = torch.empty(Cout, dtype=torch.float32, device=xc.device) if want_b else None
            work = {'flops': 2.0 * N * Ho * Wo * Cout * 9 * Cx, 'bytes': (dyc.numel() + xc.numel()) * 2}
            L.call('ewvit_conv3x3_bwd_weight', L.ptr(xc), L.ptr(dyc), L.ptr(dwf), L.ptr(dbf), 0, N, H, W, Cx,
                   Cout, stride, L.ptr(ws), L.stream(dwf), work=work)
            if ctx.needs_input_grad[1]:
                dw = dwf if Cx == Cin else dwf[:, :Cin]
                if dw.stride() != weight.stride():     # keep the parameter's layout (DDP bucket views)
                    dw = torch.empty_like(weight, dtype=torch.float32).copy_(dw)
            db = dbf
        return dx, dw, db, None


def conv3x3(x, weight, bias=None, stride=1):
    """Conv2d(kernel 3, padding 1, stride) — NCHW logical / channels-last bf16 output."""
    return Conv3x3Fn.apply(x, weight, bias, int(stride))
