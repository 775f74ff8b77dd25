"""Squeeze-excitation and stochastic-depth residual add on the ewvit kernels
(csrc/se.hip) — the MBConv block tail of the EfficientNetV2-S backbone
(torchvision SqueezeExcitation / StochasticDepth behind network/sfe.py:111-113).

SE: s = sigmoid(fc2(silu(fc1(mean_hw x)))), y = x * s.  The two HBM passes of the
forward (squeeze, excite) and of the backward (sum_hw dy*x, dx = dy*s + dsq/HW)
are ewvit kernels, and so is the fp32 [N, C] squeeze MLP: one launch forward
(fc1 + SiLU + fc2 + sigmoid), two backward (per-frame vectors; weight/bias sums)
in place of the ~15 small library/elementwise kernels of the reference block.
``bn_act_se`` takes the BatchNorm + SiLU before the SE as well: its backward folds the SE
input-gradient pass into the BatchNorm backward.
"""
import os

import torch
import torch.nn.functional as F

from . import _lib as L
from . import grads

# the depthwise BatchNorm's apply pass and the SE squeeze as one kernel when the statistics come
# from the depthwise conv (ewvit_bn_act_se_squeeze; 0: separate passes, A/B)
_BN_SQUEEZE = os.environ.get('EWVIT_BN_SQUEEZE', '1') != '0'
# the depthwise BN's backward reduction inside the SE backward's squeeze pass (ewvit_bn_se_bwd);
# EWVIT_BN_SE_FUSED=0: ewvit_se_squeeze_mlp_bwd + ewvit_bn_bwd_se (A/B)
_BN_SE_FUSED = os.environ.get('EWVIT_BN_SE_FUSED', '1') != '0'
# the BN + SE backward's dx pass folded into the depthwise conv's fused backward (SeDxLink).  Off:
# measured 2 % slower at config 2 (3834-3842 against 3908-3920 frames/s, same box,
# profiles/r06/s2/ab/se_dx_fold.log) — the transform (an exp and a reciprocal per element, three
# times per element across the row windows) and 234 VGPRs cost the depthwise backward more than
# the dz pass it removes.  EWVIT_SE_DX_FOLD=1: the A/B.
_SE_DX_FOLD = os.environ.get('EWVIT_SE_DX_FOLD', '0') == '1'


class SeDxLink:
    """MBConv's depthwise conv -> BatchNorm -> SiLU -> SE (reference network/sfe.py:111-113, the
    torchvision blocks): the BN + SE backward (BnActSEFn) computes its sums but leaves the dx pass
    to the depthwise conv's backward, which forms dz per window element from the SE output
    gradient and z (ewvit_dwconv3x3_bwd_fused_se) — the dz tensor is never written or read.
    BnActSEFn returns an unwritten placeholder for dz; the conv's backward, the only consumer of
    that gradient (the pair is built by network.efficientnet._seq), either folds it (``take``)
    or has the dx pass write it first (``materialize``)."""

    def __init__(self):
        self.dx = None          # the placeholder handed to autograd
        self.args = None        # what the dx pass needs (SimpleNamespace-like)

    def pending(self, dy):
        return self.args is not None and self.dx is not None and dy.data_ptr() == self.dx.data_ptr()

    def take(self):
        a, self.args, self.dx = self.args, None, None
        return a

    def materialize(self):
        a, dx = self.args, self.dx
        self.args = self.dx = None
        if a is None:
            return
        L.call('ewvit_bn_se_bwd_dx', L.ptr(a.dy), L.ptr(a.z), L.ptr(dx), L.dt(a.z), a.N, a.HW, a.C, L.ptr(a.gamma),
               L.ptr(a.beta), L.ptr(a.mean), L.ptr(a.invstd), a.act, L.ptr(a.s), L.ptr(a.g), L.ptr(a.row),
               L.stream(dx), work={'bytes': 3 * dx.numel() * dx.element_size()})


class _SeDxArgs:
    __slots__ = ('dy', 'z', 'gamma', 'beta', 'mean', 'invstd', 'act', 's', 'g', 'row', 'N', 'HW', 'C', 'ws')
# (the BatchNorm backward's sums taken per frame by the SE backward's squeeze kernel measured
# slower — SFE piece 14.22-14.25 -> 14.28-14.32 ms, profiles/r03/ab/se_bn_sums_ab.txt — and
# was removed: that kernel walks one frame's 49-196 rows per block, so the extra operand's loads
# land on its latency path, while the reduction pass they replace streams the whole map)


def _rows(x):
    xc = x.contiguous(memory_format=torch.channels_last)
    N, C, H, W = xc.shape
    return xc, N, H * W, C


def _ws(N, HW, C, dev):
    return torch.empty(L.load().ewvit_se_reduce_workspace(N, HW, C) // 4, dtype=torch.float32, device=dev)


def _mat(w, r, c):
    """fp32 [r, c] matrix over a 1x1 conv weight's memory (no copy for fp32 weights)."""
    return w.detach().float().reshape(r, c).contiguous()


def _vec(b):
    return None if b is None else b.detach().float().contiguous()


def _grad_like(g, p):
    """gradient in the parameter's own strides (DDP bucket views); size-1 dims' strides
    are free, so a 1x1 conv weight's channels-last gradient is a view, not a copy."""
    g = g.reshape(p.shape)
    if g.stride() == p.stride():
        return g
    if all(a == b for a, b, n in zip(g.stride(), p.stride(), p.shape) if n != 1) and g.is_contiguous():
        return g.as_strided(p.shape, p.stride())
    return torch.empty_like(p, dtype=g.dtype).copy_(g)


def _dense(o):
    """True when tensor o's layout is row-major over its non-size-1 dims."""
    exp, st = [], 1
    for n in reversed(o.shape):
        exp.append(st)
        st *= n
    return all(a == b for a, b, n in zip(o.stride(), reversed(exp), o.shape) if n != 1)


def _mat_out(p, gen, r, c, dev):
    """([r, c] fp32 matrix the kernel writes, the parameter-shaped gradient it is or None): the
    parameter's gradient slot (ewvit.grads) when its layout is [r][c] row-major."""
    o = grads.grad_out(p, gen)
    if o.dtype == torch.float32 and _dense(o):
        return o.as_strided((r, c), (c, 1)), o
    return torch.empty(r, c, dtype=torch.float32, device=dev), None


def _vec_out(p, gen, n, dev):
    if p is None:
        return None
    o = grads.grad_out(p, gen)
    return o if o.dim() == 1 and o.is_contiguous() and o.dtype == torch.float32 else torch.empty(
        n, dtype=torch.float32, device=dev)


def _track(ctx, *params):
    """Count the uses of the op's parameters (ewvit.grads) and keep them for the backward."""
    ctx.gen = grads.note_use(None)
    for p in params:
        grads.note_use(p)
    ctx.params = params


class SqueezeExciteFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        L.require_gpu(x)
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        xc, N, HW, C = _rows(x)
        Csq = w1.shape[0]
        s0 = torch.empty(N, C, dtype=torch.float32, device=x.device)
        W1, W2 = _mat(w1, Csq, C), _mat(w2, C, Csq)
        h1 = torch.empty(N, Csq, dtype=torch.float32, device=x.device)
        s = torch.empty(N, C, dtype=torch.float32, device=x.device)
        fws = torch.empty(L.load().ewvit_se_mlp_fwd_workspace(N, C, Csq) // 4, dtype=torch.float32, device=x.device)
        y = torch.empty_like(xc)
        # squeeze (mean over HW) inside the MLP's first kernel; gates + excite pass in the second
        L.call('ewvit_se_forward', L.ptr(xc), L.dt(xc), N, HW, C, L.ptr(W1), L.ptr(_vec(b1)), L.ptr(W2),
               L.ptr(_vec(b2)), Csq, L.ptr(s0), L.ptr(h1), L.ptr(s), L.ptr(y), L.ptr(fws), L.stream(y),
               work={'bytes': 3 * xc.numel() * xc.element_size()})
        ctx.save_for_backward(xc, w1, w2, s0, h1, s)
        ctx.has_b = (b1 is not None, b2 is not None)
        _track(ctx, w1, b1, w2, b2)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w1, w2, s0, h1, s = ctx.saved_tensors
        N, C, H, W = xc.shape
        HW, Csq = H * W, w1.shape[0]
        dev = xc.device
        dyc = dy.to(xc.dtype).contiguous(memory_format=torch.channels_last)
        W1, W2 = _mat(w1, Csq, C), _mat(w2, C, Csq)
        g = torch.empty(N, C, dtype=torch.float32, device=dev)
        pw1, pb1, pw2, pb2 = ctx.params
        dW1, o1 = _mat_out(pw1, ctx.gen, Csq, C, dev)
        dW2, o2 = _mat_out(pw2, ctx.gen, C, Csq, dev)
        db1 = _vec_out(pb1, ctx.gen, Csq, dev)
        db2 = _vec_out(pb2, ctx.gen, C, dev)
        mws = torch.empty(L.load().ewvit_se_mlp_bwd_workspace(N, C, Csq) // 4, dtype=torch.float32, device=dev)
        # ds = sum_hw dy * x inside the backward MLP's first kernel
        L.call('ewvit_se_squeeze_mlp_bwd', L.ptr(dyc), L.ptr(xc), L.dt(xc), N, HW, C, L.ptr(s), L.ptr(h1), L.ptr(s0),
               L.ptr(W1), L.ptr(W2), Csq, L.ptr(g), L.ptr(dW1), L.ptr(db1), L.ptr(dW2), L.ptr(db2), L.ptr(mws),
               L.stream(g), work={'bytes': 2 * xc.numel() * xc.element_size()})
        dx = torch.empty_like(xc)
        L.call('ewvit_se_scale', L.ptr(dyc), L.dt(xc), L.ptr(s), L.ptr(g), L.ptr(dx), N, HW, C, L.stream(dx),
               work={'bytes': 2 * xc.numel() * xc.element_size()})
        return dx, *_give_se(ctx, dW1, o1, db1, dW2, o2, db2)


def _give_se(ctx, dW1, o1, db1, dW2, o2, db2):
    """The SE parameters' gradients as autograd receives them (ewvit.grads.give)."""
    pw1, pb1, pw2, pb2 = ctx.params[-4:]
    g = ctx.gen
    return (grads.give(pw1, o1 if o1 is not None else _grad_like(dW1, pw1), g), grads.give(pb1, db1, g),
            grads.give(pw2, o2 if o2 is not None else _grad_like(dW2, pw2), g), grads.give(pb2, db2, g))


class BnActSEFn(torch.autograd.Function):
    """SE(act(BatchNorm(x))) in training mode — MBConv's depthwise BN + SiLU followed by its
    squeeze-excitation.  Forward: the BatchNorm statistics + apply passes, then the SE's squeeze
    MLP and excite pass (the same kernels as batch_norm_act + squeeze_excite).  Backward: the SE
    MLP backward gives the squeeze term g, and the BatchNorm backward forms its output gradient
    dy*s + g itself (ewvit_bn_bwd_se) — the SE input-gradient pass and its tensor never exist."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, momentum, eps, counter, act, w1, b1, w2, b2,
                partials=None, link=None):
        L.require_gpu(x)
        ctx.link = link
        xc, N, HW, C = _rows(x)
        M = N * HW
        dev = x.device
        x2 = torch.empty_like(xc)
        mean = torch.empty(1, C, dtype=torch.float32, device=dev)
        invstd = torch.empty_like(mean)
        Csq = w1.shape[0]
        W1, W2 = _mat(w1, Csq, C), _mat(w2, C, Csq)
        s0 = torch.empty(N, C, dtype=torch.float32, device=dev)
        h1 = torch.empty(N, Csq, dtype=torch.float32, device=dev)
        sc = torch.empty(N, C, dtype=torch.float32, device=dev)
        fws = torch.empty(L.load().ewvit_se_mlp_fwd_workspace(N, C, Csq) // 4, dtype=torch.float32, device=dev)
        y = torch.empty_like(x2)
        if partials is not None and _BN_SQUEEZE and N <= 65535:
            # BatchNorm apply + SiLU + the SE squeeze (+ the MLP's first-layer partials) in one
            # pass, then the gates + excite: 2 launches for the BN and the SE forward
            part, shifts, nrc = partials
            L.call('ewvit_bn_act_se_squeeze', L.ptr(xc), L.ptr(x2), L.dt(xc), N, HW, C, L.ptr(gamma), L.ptr(beta),
                   L.ptr(running_mean), L.ptr(running_var), float(momentum), float(eps), act, L.ptr(mean),
                   L.ptr(invstd), L.ptr(counter), L.ptr(part), L.ptr(shifts), int(nrc), L.ptr(W1), Csq, L.ptr(s0),
                   L.ptr(fws), L.stream(x2), work={'bytes': 2 * xc.numel() * xc.element_size()})
            L.call('ewvit_se_gate_excite', L.ptr(fws), L.ptr(_vec(b1)), L.ptr(W2), L.ptr(_vec(b2)), L.ptr(x2),
                   L.dt(x2), N, HW, C, Csq, L.ptr(h1), L.ptr(sc), L.ptr(y), L.stream(y),
                   work={'bytes': 2 * x2.numel() * x2.element_size()})
            ctx.save_for_backward(xc, gamma, beta, mean, invstd, x2, w1, w2, s0, h1, sc)
            ctx.cfg = (act, b1 is not None, b2 is not None)
            _track(ctx, gamma, beta, w1, b1, w2, b2)
            return y
        if partials is not None:
            # statistics summed by the depthwise conv that produced x: the apply pass only
            part, shifts, nrc = partials
            L.call('ewvit_bn_fwd_partials', L.ptr(xc), L.ptr(x2), L.dt(xc), M, C, L.ptr(gamma), L.ptr(beta),
                   L.ptr(running_mean), L.ptr(running_var), float(momentum), float(eps), act, L.ptr(mean),
                   L.ptr(invstd), L.ptr(counter), L.ptr(part), L.ptr(shifts), int(nrc), 1, L.stream(x2),
                   work={'bytes': 2 * xc.numel() * xc.element_size()})
        else:
            ws = torch.empty(L.load().ewvit_bn_workspace(M, C, 1) // 4, dtype=torch.float32, device=dev)
            L.call('ewvit_bn_fwd', L.ptr(xc), L.ptr(x2), L.dt(xc), M, C, L.ptr(gamma), L.ptr(beta),
                   L.ptr(running_mean), L.ptr(running_var), 1, float(momentum), float(eps), act, L.ptr(mean),
                   L.ptr(invstd), 1, L.ptr(counter), L.ptr(ws), L.stream(x2),
                   work={'bytes': 3 * xc.numel() * xc.element_size()})
        # squeeze + MLP hidden partials, then the gates and the excite pass in one launch
        L.call('ewvit_se_forward', L.ptr(x2), L.dt(x2), N, HW, C, L.ptr(W1), L.ptr(_vec(b1)), L.ptr(W2),
               L.ptr(_vec(b2)), Csq, L.ptr(s0), L.ptr(h1), L.ptr(sc), L.ptr(y), L.ptr(fws), L.stream(y),
               work={'bytes': 3 * x2.numel() * x2.element_size()})
        ctx.save_for_backward(xc, gamma, beta, mean, invstd, x2, w1, w2, s0, h1, sc)
        ctx.cfg = (act, b1 is not None, b2 is not None)
        _track(ctx, gamma, beta, w1, b1, w2, b2)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, gamma, beta, mean, invstd, x2, w1, w2, s0, h1, sc = ctx.saved_tensors
        act, has_b1, has_b2 = ctx.cfg
        N, C, H, W = xc.shape
        HW, M, Csq = H * W, N * H * W, w1.shape[0]
        dev = xc.device
        dyc = dy.to(xc.dtype).contiguous(memory_format=torch.channels_last)
        W1, W2 = _mat(w1, Csq, C), _mat(w2, C, Csq)
        g = torch.empty(N, C, dtype=torch.float32, device=dev)
        pg, pb, pw1, pb1, pw2, pb2 = ctx.params
        dW1, o1 = _mat_out(pw1, ctx.gen, Csq, C, dev)
        dW2, o2 = _mat_out(pw2, ctx.gen, C, Csq, dev)
        db1 = _vec_out(pb1, ctx.gen, Csq, dev)
        db2 = _vec_out(pb2, ctx.gen, C, dev)
        dx = torch.empty_like(xc)
        dg = _vec_out(pg, ctx.gen, C, dev)
        db = _vec_out(pb, ctx.gen, C, dev)
        link, ctx.link = ctx.link, None
        if _BN_SE_FUSED and C <= 4096 and L.has('ewvit_bn_se_bwd'):
            # the BN's reduction inside the SE squeeze pass: 4 launches, dy and z read once fewer
            mws = torch.empty(L.load().ewvit_bn_se_bwd_workspace(N, C, Csq) // 4, dtype=torch.float32, device=dev)
            if (link is not None and _SE_DX_FOLD and xc.dtype == torch.bfloat16 and
                    L.has('ewvit_dwconv3x3_bwd_fused_se') and ctx.needs_input_grad[0]):
                # 3 launches: the sums (and dgamma / dbeta); the dx pass is the depthwise conv's
                L.call('ewvit_bn_se_bwd', L.ptr(dyc), L.ptr(x2), L.ptr(xc), None, L.dt(xc), N, HW, C, L.ptr(gamma),
                       L.ptr(beta), L.ptr(mean), L.ptr(invstd), act, L.ptr(dg), L.ptr(db), L.ptr(sc), L.ptr(h1),
                       L.ptr(s0), L.ptr(W1), L.ptr(W2), Csq, L.ptr(g), L.ptr(dW1), L.ptr(db1), L.ptr(dW2), L.ptr(db2),
                       L.ptr(mws), L.stream(dx), work={'bytes': 3 * xc.numel() * xc.element_size()})
                off = int(L.load().ewvit_bn_se_bwd_row_offset(N, C, Csq))
                a = _SeDxArgs()
                a.dy, a.z, a.gamma, a.beta, a.mean, a.invstd, a.act = dyc, xc, gamma, beta, mean, invstd, act
                a.s, a.g, a.row, a.N, a.HW, a.C, a.ws = sc, g, mws[off:off + 2 * C], N, HW, C, mws
                link.args, link.dx = a, dx
                return (dx, grads.give(pg, dg, ctx.gen), grads.give(pb, db, ctx.gen), None, None, None, None, None,
                        None, *_give_se(ctx, dW1, o1, db1, dW2, o2, db2), None, None)
            L.call('ewvit_bn_se_bwd', L.ptr(dyc), L.ptr(x2), L.ptr(xc), L.ptr(dx), L.dt(xc), N, HW, C, L.ptr(gamma),
                   L.ptr(beta), L.ptr(mean), L.ptr(invstd), act, L.ptr(dg), L.ptr(db), L.ptr(sc), L.ptr(h1),
                   L.ptr(s0), L.ptr(W1), L.ptr(W2), Csq, L.ptr(g), L.ptr(dW1), L.ptr(db1), L.ptr(dW2), L.ptr(db2),
                   L.ptr(mws), L.stream(dx), work={'bytes': 6 * xc.numel() * xc.element_size()})
            return (dx, grads.give(pg, dg, ctx.gen), grads.give(pb, db, ctx.gen), None, None, None, None, None, None,
                    *_give_se(ctx, dW1, o1, db1, dW2, o2, db2), None, None)
        mws = torch.empty(L.load().ewvit_se_mlp_bwd_workspace(N, C, Csq) // 4, dtype=torch.float32, device=dev)
        L.call('ewvit_se_squeeze_mlp_bwd', L.ptr(dyc), L.ptr(x2), L.dt(x2), N, HW, C, L.ptr(sc), L.ptr(h1), L.ptr(s0),
               L.ptr(W1), L.ptr(W2), Csq, L.ptr(g), L.ptr(dW1), L.ptr(db1), L.ptr(dW2), L.ptr(db2), L.ptr(mws),
               L.stream(g), work={'bytes': 2 * x2.numel() * x2.element_size()})
        ws = torch.empty(L.load().ewvit_bn_workspace(M, C, 1) // 4, dtype=torch.float32, device=dev)
        L.call('ewvit_bn_bwd_se', L.ptr(dyc), L.ptr(xc), L.ptr(dx), L.dt(xc), M, C, L.ptr(gamma), L.ptr(beta),
               L.ptr(mean), L.ptr(invstd), act, L.ptr(dg), L.ptr(db), L.ptr(sc), L.ptr(g), HW, L.ptr(ws),
               L.stream(dx), work={'bytes': 5 * xc.numel() * xc.element_size()})
        return (dx, grads.give(pg, dg, ctx.gen), grads.give(pb, db, ctx.gen), None, None, None, None, None, None,
                *_give_se(ctx, dW1, o1, db1, dW2, o2, db2), None, None)


def bn_act_se(x, bn, act, se_w1, se_b1, se_w2, se_b2, partials=None, link=None):
    """SE(act(bn(x))) for a training-mode BatchNorm module `bn` (batch statistics, running
    statistics and counter updated like batch_norm_act) and the SE's 1x1 conv parameters
    (fc1 = (se_w1, se_b1), fc2 = (se_w2, se_b2)) — see BnActSEFn.  `partials` = (part,
    shifts, nrc): x's batch statistics already summed by its producer
    (ewvit.ops.dwconv3x3_bn_stats)."""
    from .bn import ACT
    if not bn.training or bn.momentum is None:
        raise ValueError('bn_act_se: training-mode BatchNorm with a momentum only')
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    counter = bn.num_batches_tracked if bn.track_running_stats else None
    return BnActSEFn.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps, counter,
                           ACT[act], se_w1, se_b1, se_w2, se_b2, partials, link)


def squeeze_excite(x, w1, b1, w2, b2):
    """torchvision SqueezeExcitation(C, Csq) with fc1 = (w1 [Csq, C, 1, 1], b1),
    fc2 = (w2 [C, Csq, 1, 1], b2), SiLU / Sigmoid: x * sigmoid(fc2(silu(fc1(avgpool(x)))))."""
    return SqueezeExciteFn.apply(x, w1, b1, w2, b2)


class ScaleAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, x, scale):
        L.require_gpu(r, x)
        rc = r.contiguous(memory_format=torch.channels_last)
        xc = x.to(rc.dtype).contiguous(memory_format=torch.channels_last)
        N = rc.shape[0]
        y = torch.empty_like(rc)
        L.call('ewvit_scale_add', L.ptr(rc), L.ptr(xc), L.dt(rc), L.ptr(scale), L.ptr(y), N, rc.numel() // N,
               L.stream(y), work={'bytes': 3 * rc.numel() * rc.element_size()})
        ctx.save_for_backward(scale)
        ctx.xdt = x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        scale, = ctx.saved_tensors
        dyc = dy.contiguous(memory_format=torch.channels_last)
        N = dyc.shape[0]
        dr = torch.empty_like(dyc)
        L.call('ewvit_scale_add', L.ptr(dyc), None, L.dt(dyc), L.ptr(scale), L.ptr(dr), N, dyc.numel() // N,
               L.stream(dr), work={'bytes': 2 * dyc.numel() * dyc.element_size()})
        return dr, dy.to(ctx.xdt), None


class DropAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, x, keep_prob):
        from .ops import _seed
        L.require_gpu(r, x)
        rc = r.contiguous(memory_format=torch.channels_last)
        xc = x.to(rc.dtype).contiguous(memory_format=torch.channels_last)
        N = rc.shape[0]
        y = torch.empty_like(rc)
        scale = torch.empty(N, dtype=torch.float32, device=r.device)
        L.call('ewvit_scale_add_drop', L.ptr(rc), L.ptr(xc), L.dt(rc), float(keep_prob), _seed(),
               L.ptr(L.rng_offset(r.device)), L.ptr(scale), L.ptr(y), N, rc.numel() // N, L.stream(y),
               work={'bytes': 3 * rc.numel() * rc.element_size()})
        ctx.save_for_backward(scale)
        ctx.xdt = x.dtype
        return y

    backward = ScaleAddFn.backward


def drop_add(r, x, drop_prob):
    """StochasticDepth(p=drop_prob, mode='row')(r) + x in one pass, the per-sample keep
    mask drawn in the kernel (counter hash of a per-call seed and the ewvit step
    counter, as ewvit dropout draws; advanced by _lib.rng_advance once per step)."""
    return DropAddFn.apply(r, x, 1.0 - float(drop_prob))


def scale_add(r, scale, x):
    """r * scale[n] + x for [N, C, H, W] tensors (scale: f32 [N], no gradient) —
    StochasticDepth(mode='row') fused with the residual add of an MBConv block."""
    return ScaleAddFn.apply(r, x, scale.float().contiguous())
