"""The MWT seperate convs on csrc/hfsep.hip (reference network/mwt.py:48-59, 84-86).

``hf_conv['seperate'][g]`` is Conv2d(3, 18, 3, padding=1) on colour g's three HF bands, the
weights shared by every DWT level (mwt.py:108): a grouped conv, 3 x (3 -> 18), 1458 MACs per
pixel.  ``seperate_conv`` runs all levels in one launch, reading the three modules' fp32
weights and biases directly, and — in training — leaves the per-level BatchNorm partial
statistics of its output for the grouped BN + ReLU that follows (network/mwt.py), so that BN
runs its apply pass only.  The backward computes the six parameter gradients (the HF input
never needs one: the frames do not require grad, SURVEY §8a note 7) in one pass over dy and x
plus a small fixed-order reduce.
"""
import os

import torch

from . import _lib as L
from . import grads
from .grads import grad_out

MACS_PER_PIXEL = 3 * 18 * 27


class SeperateConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, levels, shift, w0, w1, w2, b0, b1, b2):
        L.require_gpu(x, w0)
        params = (w0, w1, w2, b0, b1, b2)
        ctx.gen = grads.note_use(None)
        for i, p in enumerate(params):
            if ctx.needs_input_grad[3 + i]:
                grads.note_use(p)
        NL, C, H, W = x.shape
        if C not in (16, 9) or (C == 9 and W % 2) or NL % levels or x.dtype != torch.bfloat16:
            raise ValueError(f'seperate_conv: input {tuple(x.shape)} {x.dtype} (want [L*N, 16 | 9, H, W] bf16)')
        for w in (w0, w1, w2):
            if tuple(w.shape) != (18, 3, 3, 3) or w.dtype != torch.float32:
                raise ValueError(f'seperate_conv: weight {tuple(w.shape)} {w.dtype}')
        xc = x.contiguous(memory_format=torch.channels_last)
        N = NL // levels
        ws = [t.detach().contiguous() for t in params]
        y = torch.empty((NL, 64, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        ctx.cap = L.current_cap()
        with L.launch_cap(ctx.cap):
            part = shifts = sh = None
            nparts = 0
            if shift is not None:
                nparts = int(L.load().ewvit_hfsep_fwd_parts(levels, N, H, W))
                part = torch.empty(levels, nparts, 128, dtype=torch.float32, device=x.device)
                shifts = torch.empty(levels, 64, dtype=torch.float32, device=x.device)
                sh = shift.detach().float().contiguous()
            npx = NL * H * W
            L.call('ewvit_hfsep_fwd', L.ptr(xc), L.ptr(y), levels, N, H, W, C, *[L.ptr(t) for t in ws], L.ptr(sh),
                   L.ptr(part), L.ptr(shifts), nparts, L.stream(y),
                   work={'flops': 2.0 * npx * MACS_PER_PIXEL, 'bytes': npx * (C + 64) * 2.0})
        ctx.save_for_backward(xc)
        ctx.params = params
        outs = (y,) if shift is None else (y, part, shifts)
        for t in outs[1:]:
            ctx.mark_non_differentiable(t)
        return outs if shift is not None else y

    @staticmethod
    def backward(ctx, dy, *_):
        with L.launch_cap(L.bwd_cap(ctx.cap)):
            (xc,) = ctx.saved_tensors
            NL, C, H, W = xc.shape
            dyc = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            outs = []
            for i, p in enumerate(ctx.params):
                if ctx.needs_input_grad[3 + i]:
                    g = grad_out(p, ctx.gen)
                    if not g.is_contiguous():
                        g = torch.empty_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                    outs.append(g)
                else:
                    outs.append(None)
            ws = torch.empty(int(L.load().ewvit_hfsep_bwd_weight_workspace(NL, H, W)) // 4, dtype=torch.float32,
                             device=xc.device)
            npx = NL * H * W
            L.call('ewvit_hfsep_bwd_weight', L.ptr(xc), L.ptr(dyc), NL, H, W, C, *[L.ptr(t) for t in outs], L.ptr(ws),
                   L.stream(dyc), work={'flops': 2.0 * npx * MACS_PER_PIXEL, 'bytes': npx * (C + 64) * 2.0})
        return (None, None, None) + tuple(grads.give(p, g, ctx.gen) for p, g in zip(ctx.params, outs))


def seperate_conv(x, levels, convs, shift=None):
    """x [levels*N, 16 | 9, H, W] bf16 (channels-last storage; channel 3g+ci of colour g; 16:
    channels 9..15 zero, 9: W even) ->
    y [levels*N, 64, H, W] bf16 (channel 18g+o, 54..63 zero) with the three Conv2d modules'
    parameters; with ``shift`` (the concatenated BatchNorm running means, training) also
    (part [levels, nparts, 128], shifts [levels, 64], nparts) for ewvit.bn partials."""
    ws = [c.weight for c in convs]
    bs = [c.bias for c in convs]
    if shift is None:
        return SeperateConvFn.apply(x, int(levels), None, *ws, *bs)
    y, part, shifts = SeperateConvFn.apply(x, int(levels), shift, *ws, *bs)
    return y, (part, shifts, part.shape[1])


class SeperateBNReLUFn(torch.autograd.Function):
    """Training: the seperate convs + their grouped BatchNorm (per-level batch statistics,
    mwt.py:48-59, 84-86) + ReLU.  Forward: ewvit_hfsep_fwd (y and the BN partial sums) and the
    BN apply pass (ewvit_bn_fwd_partials), offering the BN's backward link to the consumer (the
    fusion conv).  Backward: when the consumer's input-gradient epilogue left the BN backward
    sums (the link) — or after the BN backward's own reduction pass (ewvit_bn_bwd_reduce) — ONE
    pass recomputes the BN backward's dx per element inside the weight-gradient pass
    (ewvit_hfsep_bn_bwd_weight): the BN's dx tensor is never written nor read back."""

    @staticmethod
    def forward(ctx, x, levels, cfg, w0, w1, w2, b0, b1, b2, gamma, beta):
        from .bn import offer_bwd_link
        running_mean, running_var, momentum, eps = cfg
        L.require_gpu(x, w0, gamma)
        params = (w0, w1, w2, b0, b1, b2)
        ctx.gen = grads.note_use(None)
        for i, p in enumerate(params):
            if ctx.needs_input_grad[3 + i]:
                grads.note_use(p)
        NL, C, H, W = x.shape
        if C not in (16, 9) or (C == 9 and W % 2) or NL % levels or x.dtype != torch.bfloat16 or gamma.numel() != 64:
            raise ValueError(f'seperate_conv_bn_relu: input {tuple(x.shape)} {x.dtype}, {gamma.numel()} BN channels')
        xc = x.contiguous(memory_format=torch.channels_last)
        N = NL // levels
        ws = [t.detach().contiguous() for t in params]
        dev = x.device
        y = torch.empty((NL, 64, H, W), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        z = torch.empty_like(y)
        mean = torch.empty(levels, 64, dtype=torch.float32, device=dev)
        invstd = torch.empty_like(mean)
        ctx.cap = L.current_cap()
        with L.launch_cap(ctx.cap):
            nparts = int(L.load().ewvit_hfsep_fwd_parts(levels, N, H, W))
            part = torch.empty(levels, nparts, 128, dtype=torch.float32, device=dev)
            shifts = torch.empty(levels, 64, dtype=torch.float32, device=dev)
            sh = running_mean.detach().float().contiguous()
            npx = NL * H * W
            L.call('ewvit_hfsep_fwd', L.ptr(xc), L.ptr(y), levels, N, H, W, C, *[L.ptr(t) for t in ws], L.ptr(sh),
                   L.ptr(part), L.ptr(shifts), nparts, L.stream(y),
                   work={'flops': 2.0 * npx * MACS_PER_PIXEL, 'bytes': npx * (C + 64) * 2.0})
            L.call('ewvit_bn_fwd_partials', L.ptr(y), L.ptr(z), L.BF16, npx, 64, L.ptr(gamma), L.ptr(beta),
                   L.ptr(running_mean), L.ptr(running_var), float(momentum), float(eps), 1, L.ptr(mean),
                   L.ptr(invstd), None, L.ptr(part), L.ptr(shifts), nparts, levels, L.stream(z),
                   work={'bytes': 2 * y.numel() * 2})
        ctx.save_for_backward(xc, y, mean, invstd, gamma, beta)
        ctx.params, ctx.levels = params, levels
        ctx.bnlink = offer_bwd_link(z, y, mean, invstd, gamma, beta, 1, None, levels)
        return z

    @staticmethod
    def backward(ctx, dz):
        from .bn import fold_bwd_partials
        with L.launch_cap(L.bwd_cap(ctx.cap)):
            xc, y, mean, invstd, gamma, beta = ctx.saved_tensors
            levels = ctx.levels
            NL, C, H, W = xc.shape
            N = NL // levels
            dzc = dz.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            pr = ctx.bnlink.partials_for(dzc) if ctx.bnlink is not None else None
            ctx.bnlink = None
            outs = []
            for i, p in enumerate(ctx.params):
                if ctx.needs_input_grad[3 + i]:
                    g = grad_out(p, ctx.gen)
                    if not g.is_contiguous():
                        g = torch.empty_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                    outs.append(g)
                else:
                    outs.append(None)
            dg = torch.empty(64, dtype=torch.float32, device=xc.device) if ctx.needs_input_grad[9] else None
            db = torch.empty(64, dtype=torch.float32, device=xc.device) if ctx.needs_input_grad[10] else None
            npx = NL * H * W
            work = {'flops': 2.0 * npx * MACS_PER_PIXEL, 'bytes': npx * (C + 64 + 64) * 2.0}
            if pr is not None:
                part, nrc = fold_bwd_partials(pr[0], pr[1], levels, 64)
            else:
                # no epilogue sums (the consumer took no link): the BN backward's reduction pass
                # alone; the dx pass still runs inside the weight gradient
                nrc = int(L.load().ewvit_bn_bwd_reduce_rows(npx, 64, levels))
                part = torch.empty(levels * nrc * 128, dtype=torch.float32, device=xc.device)
                L.call('ewvit_bn_bwd_reduce', L.ptr(dzc), L.ptr(y), L.BF16, npx, 64, L.ptr(gamma), L.ptr(beta),
                       L.ptr(mean), L.ptr(invstd), 1, levels, L.ptr(part), L.stream(dzc),
                       work={'bytes': 2 * y.numel() * 2})
                part, nrc = fold_bwd_partials(part, nrc, levels, 64)
            ws = torch.empty(int(L.load().ewvit_hfsep_bn_bwd_weight_workspace(levels, N, H, W)) // 4,
                             dtype=torch.float32, device=xc.device)
            L.call('ewvit_hfsep_bn_bwd_weight', L.ptr(xc), L.ptr(y), L.ptr(dzc), levels, N, H, W, C, L.ptr(mean),
                   L.ptr(invstd), L.ptr(gamma), L.ptr(beta), L.ptr(part), nrc, *[L.ptr(t) for t in outs],
                   L.ptr(dg), L.ptr(db), L.ptr(ws), L.stream(dzc), work=work)
        return (None, None, None) + tuple(grads.give(p, g, ctx.gen) for p, g in zip(ctx.params, outs)) + (dg, db)


def seperate_conv_bn_relu(x, levels, convs, cat, momentum, eps):
    """Training: relu(BN(seperate_conv(x))) with the grouped BN parameters `cat` = (weight, bias,
    running_mean, running_var) [64] (the three modules' tensors + identity padding); the running
    statistics in `cat` are updated in place (the caller copies them back to the modules)."""
    w, b, rm, rv = cat
    return SeperateBNReLUFn.apply(x, int(levels), (rm, rv, momentum, eps), *[c.weight for c in convs],
                                  *[c.bias for c in convs], w, b)


_ON = os.environ.get('EWVIT_HFSEP', '1') != '0'      # 0: the block-diagonal dense conv (A/B)


def applies(x, convs):
    """The shape class of seperate_conv: bf16 16-channel (or 9-channel, W even) HF input on the
    GPU, three Conv2d(3, 18, 3, padding=1) with biases, no hooks."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] in (16, 9)
            and not (x.shape[1] == 9 and x.shape[3] % 2) and convs_apply(x.shape[3], convs))


# the 9 real band channels in HBM (the kernels zero-pad K in LDS; 0: the 16-channel layout, A/B)
HF9 = os.environ.get('EWVIT_HF9', '1') != '0'


def convs_apply(W, convs):
    """The module / width part of applies(): whether a W-wide HF input of these three convs takes
    the hfsep kernels (decidable before the DWT front end writes the input)."""
    return (_ON and W <= 200
            and len(convs) == 3 and all(
                type(c) is torch.nn.Conv2d and tuple(c.weight.shape) == (18, 3, 3, 3) and c.bias is not None
                and c.stride == (1, 1) and c.padding == (1, 1) and c.dilation == (1, 1) and c.groups == 1
                and c.weight.dtype == torch.float32 and not (c._forward_hooks or c._forward_pre_hooks)
                for c in convs))
