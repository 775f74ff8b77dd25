"""BatchNorm2d fused with its activation on the ewvit kernels (csrc/batchnorm.hip).

Replaces ``nn.BatchNorm2d`` + ``nn.ReLU`` (MWT conv stack, network/mwt.py:23-72)
and ``nn.BatchNorm2d`` + ``nn.SiLU`` (EfficientNetV2-S Conv2dNormActivation) on
channels-last tensors; training mode uses batch statistics and updates the
module's running statistics in place like ``F.batch_norm``.  ``groups`` > 1
normalises consecutive equal batch slices with their own statistics (one
launch for the MWT's per-level calls of its shared BatchNorms).
"""
import os
import threading
import weakref

import torch

from . import _lib as L
from . import grads

ACT = {None: 0, 'none': 0, 'relu': 1, 'silu': 2}

# BatchNorm backward statistics summed by the op that produces the BN output's gradient
# (EWVIT_BN_BWD_LINK=0: every BN backward runs its own reduction pass, A/B)
_BWD_LINK = os.environ.get('EWVIT_BN_BWD_LINK', '1') != '0'
# the most partial rows a linked producer may leave (the dx pass reads them all per block).
# Links over bigger maps (the MWT's 2.4 M-row convs, partials folded) measured slower — the
# input-gradient epilogue's BN-input reads under the capped walk cost more than the reduction
# pass they replace (MWT capped 14.0 -> 15.6 ms) — so those BNs reduce themselves.
# 128 since round 6 (the 28^2 backbone maps now reduce themselves): 3957-3963 against 3925-3935
# frames/s at 512, 64 3960-3962, 32 3948-3950, 2048 / 8192 3888-3893 / 3874-3877, no links 3794-3798
# (profiles/r06/s2/ab/bwd_link_rows.log)
BWD_LINK_MAX_ROWS = int(os.environ.get('EWVIT_BWD_LINK_MAX_ROWS', '128'))


class BwdStatsLink:
    """The reduction pass of a training-mode BatchNorm backward, done by the kernel that
    produces the gradient of the BN's output — the input gradient of the op that consumed it
    (ewvit_conv2d_bwd_data_bn, ewvit_dwconv3x3_bwd_data_bn).  The BN forward offers a link for
    its output (`offer`); the consuming op takes it in its forward (`take_bwd_link`); its
    backward `fulfil`s it with the partial sums and the gradient tensor it produced.  The BN
    backward uses the partials only if the gradient it receives IS that tensor, unmodified
    (`partials_for`): a second consumer's gradient added by autograd gives a new tensor (the
    link holds a reference to the produced one, so autograd cannot accumulate into it in
    place) and the BN runs its own reduction."""
    __slots__ = ('key', 'yref', 'x', 'mean', 'invstd', 'gamma', 'beta', 'act', 'rscale', 'groups', 'part', 'nrc',
                 'dx', 'ver')

    def __init__(self, y, x, mean, invstd, gamma, beta, act, rscale=None, groups=1):
        self.key = (y.data_ptr(), tuple(y.shape), y.dtype)
        # the offer holds only while y lives: after y is freed another tensor can take its
        # address and shape, and must not pick up this BatchNorm's link
        self.yref = weakref.ref(y)
        self.x, self.mean, self.invstd, self.gamma, self.beta = x, mean, invstd, gamma, beta
        self.act, self.rscale, self.groups = act, rscale, groups
        self.part = self.dx = None
        self.nrc = 0
        self.ver = -1

    def fulfil(self, part, nrc, dx):
        self.part, self.nrc, self.dx, self.ver = part, int(nrc), dx, dx._version

    def partials_for(self, dy):
        """(part, nrc) when dy is the fulfilling op's gradient tensor, else None; releases
        the link's references either way."""
        dx, part, nrc, ver = self.dx, self.part, self.nrc, self.ver
        self.dx = self.part = self.x = None
        if (dx is None or dy.data_ptr() != dx.data_ptr() or dy.shape != dx.shape or dy.dtype != dx.dtype
                or dy.stride() != dx.stride() or dx._version != ver):
            return None
        return part, nrc


# the offered link, per thread (nn.DataParallel replicas run in threads, reference
# train.py:249-251): a replica's consumer must only ever see its own BatchNorm's offer
_tls = threading.local()
_zeros = {}


def fold_bwd_partials(part, nrc, groups, C):
    """(part, nrc) with at most BWD_LINK_MAX_ROWS partial rows per group: a producer over a big
    map (the MWT's 2.4 M-row convs: 6272 m-tiles per level) leaves more than the dx pass should
    finalise from per block, so one launch folds them in a fixed order (ewvit_bn_fold_partials)."""
    if nrc <= BWD_LINK_MAX_ROWS:
        return part, nrc
    nout = 256
    dev = part.device
    z = _zeros.get((dev, C))
    if z is None:
        z = _zeros[(dev, C)] = torch.zeros(C, dtype=torch.float32, device=dev)
    out = torch.empty(groups * nout, 2 * C, dtype=torch.float32, device=dev)
    sh = torch.empty(groups, C, dtype=torch.float32, device=dev)
    L.call('ewvit_bn_fold_partials', L.ptr(part), nrc, L.ptr(z), L.ptr(out), nout, L.ptr(sh), C, groups,
           L.stream(part), work={'bytes': part.numel() * 4})
    return out, nout


def offer_bwd_link(y, x, mean, invstd, gamma, beta, act, rscale=None, groups=1):
    """Offer the backward statistics of the BN that produced y (4-D NHWC bf16; `groups`
    consecutive batch slices with their own statistics) to y's consumer; returns the link
    (kept by the BN's backward), or None."""
    if not (_BWD_LINK and y.dim() == 4 and y.dtype == torch.bfloat16 and x.dtype == torch.bfloat16):
        _tls.offered = None
        return None
    _tls.offered = BwdStatsLink(y, x, mean, invstd, gamma, beta, act, rscale, groups)
    return _tls.offered


def take_bwd_link(x, grouped=True, scaled=True):
    """The link offered for x (the consumer's input), if any; one taker.  A consumer whose
    backward kernel sums over whole maps only (no per-group partial rows) passes
    grouped=False, one that cannot apply a per-frame row scale (the drop-path factor of
    BNDropAddFn) scaled=False: such links are left to the BatchNorm's own reduction pass."""
    link = getattr(_tls, 'offered', None)
    if link is not None and link.key == (x.data_ptr(), tuple(x.shape), x.dtype):
        _tls.offered = None
        if link.yref() is not None and link.x is not None and (grouped or link.groups == 1) and \
                (scaled or link.rscale is None):
            return link
    return None


def _rows(x):
    """[N, C, H, W] channels-last (or [N, C]) -> contiguous NHWC storage, M rows."""
    C = x.shape[1]
    xc = x.contiguous(memory_format=torch.channels_last) if x.dim() == 4 else x.contiguous()
    return xc, xc.numel() // C, C


class BatchNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, training, momentum, eps, act, groups, counter,
                partials=None):
        ctx.cap = L.current_cap()          # a stream branch's workgroup cap (ewvit._lib.grid_cap)
        with L.launch_cap(ctx.cap):
            return BatchNormActFn._forward(ctx, x, weight, bias, running_mean, running_var, training, momentum,
                                           eps, act, groups, counter, partials)

    @staticmethod
    def _forward(ctx, x, weight, bias, running_mean, running_var, training, momentum, eps, act, groups, counter,
                 partials):
        L.require_gpu(x)
        xc, M, C = _rows(x)
        if M % groups:
            raise ValueError(f'batch_norm_act: {M} rows not divisible into {groups} groups')
        y = torch.empty_like(xc)
        mean = torch.empty(groups, C, dtype=torch.float32, device=x.device) if training else None
        invstd = torch.empty_like(mean) if training else None
        if partials is not None:
            # statistics already summed by the producing conv's epilogue: apply pass only
            part, shifts, nrc = partials
            if not training:
                raise ValueError('batch_norm_act: partial statistics need training mode')
            L.call('ewvit_bn_fwd_partials', L.ptr(xc), L.ptr(y), L.dt(xc), M, C, L.ptr(weight), L.ptr(bias),
                   L.ptr(running_mean), L.ptr(running_var), float(momentum), float(eps), act, L.ptr(mean),
                   L.ptr(invstd), L.ptr(counter), L.ptr(part), L.ptr(shifts), int(nrc), groups, L.stream(y),
                   work={'bytes': 2 * xc.numel() * xc.element_size()})
        else:
            ws = torch.empty(L.load().ewvit_bn_workspace(M, C, groups) // 4, dtype=torch.float32, device=x.device)
            L.call('ewvit_bn_fwd', L.ptr(xc), L.ptr(y), L.dt(xc), M, C, L.ptr(weight), L.ptr(bias),
                   L.ptr(running_mean), L.ptr(running_var), int(training), float(momentum), float(eps), act,
                   L.ptr(mean), L.ptr(invstd), groups, L.ptr(counter if training else None), L.ptr(ws),
                   L.stream(y), work={'bytes': (2 + int(training)) * xc.numel() * xc.element_size()})
        if training:
            ctx.save_for_backward(xc, weight, bias, mean, invstd)
            ctx.gen = grads.note_use(weight)
            grads.note_use(bias)
            ctx.params = (weight, bias)
        ctx.cfg = (training, act, M, C, groups)
        ctx.bnlink = offer_bwd_link(y, xc, mean, invstd, weight, bias, act, None, groups) if training else None
        return y

    @staticmethod
    def backward(ctx, dy):
        with L.launch_cap(L.bwd_cap(ctx.cap)):
            return BatchNormActFn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        training, act, M, C, groups = ctx.cfg
        if not training:
            raise RuntimeError('ewvit BatchNorm: backward through eval-mode statistics is not implemented')
        xc, weight, bias, mean, invstd = ctx.saved_tensors
        dyc = dy.to(xc.dtype)
        dyc = dyc.contiguous(memory_format=torch.channels_last) if dyc.dim() == 4 else dyc.contiguous()
        dx = torch.empty_like(xc)
        wp, bp = ctx.params
        dg = _affine_grad(wp, ctx.gen, C, dy.device)
        db = _affine_grad(bp, ctx.gen, C, dy.device)
        pr = ctx.bnlink.partials_for(dyc) if ctx.bnlink is not None else None
        ctx.bnlink = None
        if pr is not None:
            # the reduction was summed by the kernel that produced dy: the dx pass only
            L.call('ewvit_bn_bwd_partials', L.ptr(dyc), L.ptr(xc), L.ptr(dx), L.dt(xc), M, C, L.ptr(weight),
                   L.ptr(bias), L.ptr(mean), L.ptr(invstd), act, L.ptr(dg), L.ptr(db), None, 1, L.ptr(pr[0]), pr[1],
                   groups, L.stream(dx), work={'bytes': 3 * xc.numel() * xc.element_size()})
            return dx, grads.give(wp, dg, ctx.gen), grads.give(bp, db, ctx.gen), *(None,) * 9
        ws = torch.empty(L.load().ewvit_bn_workspace(M, C, groups) // 4, dtype=torch.float32, device=dy.device)
        L.call('ewvit_bn_bwd', L.ptr(dyc), L.ptr(xc), L.ptr(dx), L.dt(xc), M, C, L.ptr(weight), L.ptr(bias),
               L.ptr(mean), L.ptr(invstd), act, L.ptr(dg), L.ptr(db), 0, groups, L.ptr(ws), L.stream(dx),
               work={'bytes': 5 * xc.numel() * xc.element_size()})
        return dx, grads.give(wp, dg, ctx.gen), grads.give(bp, db, ctx.gen), *(None,) * 9


def _affine_grad(p, gen, C, dev):
    """The [C] fp32 output for a BatchNorm affine parameter's gradient (its gradient slot when it
    has one, ewvit.grads), or None without the parameter."""
    if p is None:
        return None
    g = grads.grad_out(p, gen)
    return g if g.dim() == 1 and g.is_contiguous() and g.dtype == torch.float32 else torch.empty(C, dtype=torch.float32, device=dev)


def batch_norm_act(x, bn, act=None, training=None, groups=1, partials=None):
    """Apply BatchNorm module `bn` (its parameters, buffers, eps, momentum) and the
    activation to x in one fused pass; updates bn's running stats and counter
    (once per statistics group, as `groups` separate module calls would).
    `partials` = (part, shifts, nrc) from ewvit.conv.conv2d_bn_stats: the batch
    statistics were summed by the conv's epilogue (training)."""
    training = bn.training if training is None else training
    if bn.momentum is None:
        raise NotImplementedError('cumulative-average BatchNorm (momentum=None) is not used by the model')
    counter = bn.num_batches_tracked if training and bn.track_running_stats else None
    return batch_norm_act_params(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, training,
                                 bn.momentum, bn.eps, act, groups, counter, partials)


def batch_norm_act_params(x, weight, bias, running_mean, running_var, training, momentum, eps, act=None,
                          groups=1, counter=None, partials=None):
    """`counter`: an int64 device tensor (a module's num_batches_tracked) the
    forward kernel increments by `groups` in training, or None."""
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    if not training:
        groups = 1
    if counter is not None and (counter.dtype != torch.int64 or counter.device != x.device):
        raise ValueError('batch_norm_act: counter must be an int64 tensor on the input device')
    return BatchNormActFn.apply(x, weight, bias, running_mean, running_var, bool(training), momentum, eps,
                                ACT[act], int(groups), counter, partials)


class BNDropAddFn(torch.autograd.Function):
    """y = BatchNorm(x) * scale[n] + skip (StochasticDepth(row) drawn in the kernel),
    training mode, one group: the MBConv block tail in one pass each way."""
    @staticmethod
    def forward(ctx, x, skip, weight, bias, running_mean, running_var, momentum, eps, counter, keep, partials,
                link=None):
        from .ops import _seed
        L.require_gpu(x, skip)
        xc, M, C = _rows(x)
        sk = skip.to(xc.dtype).contiguous(memory_format=torch.channels_last)
        N = xc.shape[0]
        y = torch.empty_like(xc)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        scale = torch.empty(N, dtype=torch.float32, device=x.device)
        if partials is not None:
            part, shifts, nrc = partials
            ws = None
        else:
            part = shifts = None
            nrc = 0
            ws = torch.empty(L.load().ewvit_bn_workspace(M, C, 1) // 4, dtype=torch.float32, device=x.device)
        L.call('ewvit_bn_fwd_drop_add', L.ptr(xc), L.ptr(y), L.dt(xc), M, C, L.ptr(weight), L.ptr(bias),
               L.ptr(running_mean), L.ptr(running_var), float(momentum), float(eps), L.ptr(mean), L.ptr(invstd),
               L.ptr(counter), L.ptr(part), L.ptr(shifts), int(nrc), L.ptr(sk), M // N, float(keep), _seed(),
               L.ptr(L.rng_offset(x.device)), L.ptr(scale), L.ptr(ws), L.stream(y),
               work={'bytes': (3 + int(partials is None)) * xc.numel() * xc.element_size()})
        ctx.save_for_backward(xc, weight, bias, mean, invstd, scale)
        ctx.gen = grads.note_use(weight)
        grads.note_use(bias)
        ctx.params = (weight, bias)
        ctx.cfg = (M, C, M // N, skip.dtype)
        ctx.link = link if link is not None and link.armed else None
        ctx.bnlink = offer_bwd_link(y, xc, mean, invstd, weight, bias, 0, scale)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, weight, bias, mean, invstd, scale = ctx.saved_tensors
        M, C, HW, sdt = ctx.cfg
        dyc = dy.to(xc.dtype).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(xc)
        wp, bp = ctx.params
        dg = _affine_grad(wp, ctx.gen, C, dy.device)
        db = _affine_grad(bp, ctx.gen, C, dy.device)
        pr = ctx.bnlink.partials_for(dyc) if ctx.bnlink is not None else None
        ctx.bnlink = None
        if pr is not None:
            # g = dy * scale[n] summed by the next conv's input-gradient epilogue: dx pass only
            L.call('ewvit_bn_bwd_partials', L.ptr(dyc), L.ptr(xc), L.ptr(dx), L.dt(xc), M, C, L.ptr(weight),
                   L.ptr(bias), L.ptr(mean), L.ptr(invstd), 0, L.ptr(dg), L.ptr(db), L.ptr(scale), HW, L.ptr(pr[0]),
                   pr[1], 1, L.stream(dx), work={'bytes': 3 * xc.numel() * xc.element_size()})
        else:
            ws = torch.empty(L.load().ewvit_bn_workspace(M, C, 1) // 4, dtype=torch.float32, device=dy.device)
            L.call('ewvit_bn_bwd_scaled', L.ptr(dyc), L.ptr(xc), L.ptr(dx), L.dt(xc), M, C, L.ptr(weight),
                   L.ptr(bias), L.ptr(mean), L.ptr(invstd), L.ptr(dg), L.ptr(db), L.ptr(scale), HW, L.ptr(ws),
                   L.stream(dx), work={'bytes': 5 * xc.numel() * xc.element_size()})
        if ctx.link is not None:
            # the skip gradient goes to the block's first conv (ewvit.conv.SkipLink), which
            # adds it to its input gradient in the dgrad epilogue
            ctx.link.grad = dy
            dskip = None
        else:
            dskip = dy.to(sdt)
        return dx, dskip, grads.give(wp, dg, ctx.gen), grads.give(bp, db, ctx.gen), *(None,) * 8


def batch_norm_drop_add(x, bn, skip, drop_prob, partials=None, link=None):
    """StochasticDepth(p=drop_prob, mode='row')(bn(x)) + skip in one pass (training):
    the keep mask is drawn in the kernel (ewvit dropout's counter hash of a per-call
    seed and the step counter); `partials` as in batch_norm_act."""
    if bn.momentum is None or not bn.training:
        raise ValueError('batch_norm_drop_add: training-mode BatchNorm with a momentum only')
    counter = bn.num_batches_tracked if bn.track_running_stats else None
    return BNDropAddFn.apply(x, skip, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                             counter, 1.0 - float(drop_prob), partials, link)
