"""Dense Conv2d (kernel 1|3, pad k/2, stride 1|2, bias) on the ewvit implicit-GEMM
kernels (csrc/conv.hip) — the MWT conv stack of network/mwt.py:23-72 and the
backbone's dense convs.

Activations are channels-last bf16 (the MFMA operand type); weights stay fp32
master parameters and are packed to bf16 [Cout][k*k][Cin] each call — or, inside
``packed()`` (the training step), once per step for all convs by one launch.  An input
may carry zero-padded channels (Cin_x > weight.shape[1]): the pack fills those
weight rows with zeros, so they contribute exactly nothing and receive no
gradient.

``levels > 1`` reads a level-major input ``z [levels*N, C, H, W]`` as the
channel concatenation ``cat(z.chunk(levels), dim=1)`` ([N, levels*C, H, W], the
multiscale fusion input of mwt.py:112) through the kernels' grouped layout, and
returns the input gradient in z's layout — the concatenation is never built.
"""
import contextlib
import ctypes
import os
import threading
import weakref

import torch

from . import _lib as L
from . import bn as bnmod
from . import defer as _defer
from . import grads
from .grads import grad_out

# ---- step-wide weight packing: every conv weight the model used is packed by ONE
# multi-tensor launch per 32 weights at the start of a training step (`packed()`),
# into persistent bf16 buffers, instead of one pack launch per conv call.
_registry = {}      # id(weight) -> {'ref', 'cin_pad', 'wp', 'wpt', 'bwd'}
# per thread (nn.DataParallel replicas run in threads, reference train.py:249-251): the
# `packed()` scope and the offered skip link
_tls = threading.local()


class SkipLink:
    """Folds a residual block's skip gradient into its first conv's input gradient.
    The block offers the link for its input x (`offer`); the conv whose input IS x takes it
    in forward (`armed`); in backward the block tail (ewvit.bn.BNDropAddFn) leaves dy in
    `grad` instead of returning it, and the conv's dgrad adds it in its epilogue — no
    separate accumulation add for x."""
    __slots__ = ('key', 'armed', 'grad')

    def __init__(self, x):
        self.key = (x.data_ptr(), tuple(x.shape), x.dtype)
        self.armed = False
        self.grad = None


grid_cap = L.grid_cap            # (ewvit._lib: the big-grid workgroup cap of a stream branch)


def offer_skip_link(x):
    _tls.offered = SkipLink(x)
    return _tls.offered


def clear_skip_link():
    _tls.offered = None


def _take_link(x):
    link = getattr(_tls, 'offered', None)
    if link is not None and link.key == (x.data_ptr(), tuple(x.shape), x.dtype):
        _tls.offered = None
        link.armed = True
        return link
    return None


def _register(weight, cin_pad, bwd):
    e = _registry.get(id(weight))
    if e is not None and e['ref']() is weight and e['cin_pad'] == cin_pad:
        e['bwd'] = e['bwd'] or bwd
        return
    _registry[id(weight)] = {'ref': weakref.ref(weight), 'cin_pad': cin_pad, 'wp': None, 'wpt': None, 'bwd': bwd}


def prepack():
    """Pack every registered conv weight into its persistent buffers (allocated on
    first use); Conv2dFn reads them while `packed()` is active."""
    items = []
    for key in list(_registry):
        e = _registry[key]
        w = e['ref']()
        if w is None or not w.is_cuda or w.dtype != torch.float32:
            del _registry[key]
            continue
        Cout, k = w.shape[0], w.shape[2]
        if e['wp'] is None or e['wp'].device != w.device:
            e['wp'] = torch.empty((Cout, k * k, e['cin_pad']), dtype=torch.bfloat16, device=w.device)
        if e['bwd'] and (e['wpt'] is None or e['wpt'].device != w.device):
            e['wpt'] = torch.empty((e['cin_pad'], k * k, Cout), dtype=torch.bfloat16, device=w.device)
        s_co, s_ci, s_kh, s_kw = w.stride()
        if s_kh != k * s_kw:
            e['wp'] = None          # not packable in place: this weight is packed per call
            continue
        items.append((w, e, (s_co, s_ci, s_kw)))
    if not items:
        return
    stream = L.stream(items[0][0])
    for i in range(0, len(items), L.PACK_MAX):
        ch = items[i:i + L.PACK_MAX]
        n = len(ch)
        vp = ctypes.c_void_p * n
        i64 = ctypes.c_int64 * n
        L.call('ewvit_conv2d_pack_weights', n, vp(*[w.data_ptr() for w, _, _ in ch]),
               i64(*[st[0] for _, _, st in ch]), i64(*[st[1] for _, _, st in ch]), i64(*[st[2] for _, _, st in ch]),
               vp(*[e['wp'].data_ptr() for _, e, _ in ch]),
               vp(*[(e['wpt'].data_ptr() if e['bwd'] else None) for _, e, _ in ch]),
               i64(*[w.shape[0] for w, _, _ in ch]), i64(*[w.shape[1] for w, _, _ in ch]),
               i64(*[e['cin_pad'] for _, e, _ in ch]), (ctypes.c_int * n)(*[w.shape[2] for w, _, _ in ch]),
               stream, work={'bytes': sum(w.numel() * 8.0 for w, _, _ in ch)})


@contextlib.contextmanager
def packed():
    """Scope of one forward(+backward) with the weights fixed: packs all registered
    conv weights once on entry; convs inside read the packs."""
    prepack()
    prev = getattr(_tls, 'active', False)
    _tls.active = True
    try:
        yield
    finally:
        _tls.active = prev


def _cached_pack(weight, cin_pad, bwd):
    if not getattr(_tls, 'active', False):
        return None
    e = _registry.get(id(weight))
    if e is None or e['ref']() is not weight or e['cin_pad'] != cin_pad or e['wp'] is None or \
            (bwd and e['wpt'] is None):
        return None
    return e['wp'], (e['wpt'] if bwd else None)


def _pack(weight, cin_pad, fwd=True, bwd=False):
    """bf16 packs of the fp32 weight (read in its own memory format): the fwd
    layout [Cout][k*k][cin_pad] and/or the bwd_data layout [cin_pad][k*k][Cout],
    one launch."""
    Cout, Cin, k = weight.shape[0], weight.shape[1], weight.shape[2]
    w = weight.detach()
    if w.dtype != torch.float32:
        w = w.float()
    s_co, s_ci, s_kh, s_kw = w.stride()
    if s_kh != k * s_kw:
        w = w.contiguous()
        s_co, s_ci, s_kh, s_kw = w.stride()
    wp = torch.empty((Cout, k * k, cin_pad), dtype=torch.bfloat16, device=w.device) if fwd else None
    wpt = torch.empty((cin_pad, k * k, Cout), dtype=torch.bfloat16, device=w.device) if bwd else None
    L.call('ewvit_conv2d_pack_weight', L.ptr(w), s_co, s_ci, s_kw, L.ptr(wp), L.ptr(wpt), Cout, Cin, cin_pad, k,
           L.stream(w))
    return wp, wpt


def _bn_link_plan(bl, xc, xdt, levels, N, H, W, Cx, Cout, k, stride, skip):
    """(groups, rows per group's slice, partial rows per group, channels per group) when this
    conv's input gradient can sum the backward statistics of the BatchNorm that produced its
    input (link `bl`), else None.  The BN's groups are either the input's levels (the level-
    major input read as a channel concatenation: channel groups of dx) or equal row slices of a
    plain input (per-level statistics of the MWT's shared BatchNorms); 128-row m-tiles."""
    if bl is None or xdt != torch.bfloat16 or bl.x.shape != xc.shape:
        return None
    tiles = int(L.load().ewvit_conv2d_bwd_bn_rows(N, H, W, Cx, Cout, k, stride))
    if tiles <= 0 or (skip is not None and levels > 1):
        return None
    if tiles > bnmod.BWD_LINK_MAX_ROWS * (levels if levels > 1 else 1):
        return None
    if skip is not None and not L.load().ewvit_conv2d_bwd_data_add_ok(N, H, W, Cx, Cout, k, stride):
        return None
    if levels > 1:
        if bl.groups != levels:
            return None
        return levels, 0, tiles, Cx // levels
    M = N * H * W
    if bl.groups > 1 and (M % bl.groups or (M // bl.groups) % 128):
        return None
    return bl.groups, (M // bl.groups if bl.groups > 1 else 0), tiles // bl.groups, Cx


def _bn_link_win(bl, xc, xdt, levels, N, H, W, Cx, Cout, k, stride, skip):
    """(row-group rows, partial rows) when the windowed input gradient takes the backward sums of
    the BatchNorm that produced this conv's plain input (hf_conv['fusion']'s 64-channel input:
    the seperate BNs, per-level statistics over slices of whole images; one partial row per
    16 x 16 block), else None."""
    if (bl is None or not _BN_BWD_EPI or levels != 1 or skip is not None or bl.rscale is not None
            or xdt != torch.bfloat16 or bl.x.shape != xc.shape or k != 3 or stride != 1):
        return None
    M = N * H * W
    if bl.groups > 1 and M % bl.groups:
        return None
    grows = M // bl.groups if bl.groups > 1 else 0
    if not L.has('ewvit_conv2d_bwd_bn_win_rows'):
        return None
    rows = int(L.load().ewvit_conv2d_bwd_bn_win_rows(N, H, W, Cx, Cout, k, stride, Cx, 0, grows))
    return (grows, rows) if rows > 0 else None


class Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, levels, bn_stats=None):
        L.require_gpu(x, weight)
        ctx.gen = grads.note_use(weight if ctx.needs_input_grad[1] else None)
        if ctx.needs_input_grad[2]:
            grads.note_use(bias)
        ctx.link = _take_link(x) if levels == 1 else None
        # the backward statistics of the BatchNorm that produced x, summed by the dgrad epilogue
        ctx.bnlink = bnmod.take_bwd_link(x) if ctx.needs_input_grad[0] else None
        NL, Cz, H, W = x.shape
        if NL % levels:
            raise ValueError(f'conv2d: batch {NL} is not a multiple of levels={levels}')
        N, Cx = NL // levels, Cz * levels
        Cout, Cin, k = weight.shape[0], weight.shape[1], weight.shape[2]
        if Cx < Cin or weight.shape[3] != k or k not in (1, 3) or (levels > 1 and Cx != Cin):
            raise ValueError(f'conv2d: input {tuple(x.shape)} (levels={levels}), weight {tuple(weight.shape)}')
        xc = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gc, gs = (Cz, N * H * W * Cz) if levels > 1 else (0, 0)
        bwd = ctx.needs_input_grad[0]
        # per-tap input channels of the fwd pack: Cx, or Cx padded to 64 when the LDS-DMA
        # kernel runs a non-multiple-of-64 input with zero lanes (wpt shares the rows)
        cp = Cx if levels > 1 else int(L.load().ewvit_conv2d_fwd_pack_cin(N, H, W, Cx, Cout, k, stride))
        cached = _cached_pack(weight, cp, bwd) if weight.dtype == torch.float32 else None
        if cached is None:
            wp, wpt = _pack(weight, cp, True, bwd)
            if weight.dtype == torch.float32:
                _register(weight, cp, bwd)
        else:
            wp, wpt = cached
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        b = bias.detach().float().contiguous() if bias is not None else None
        # algorithmic work over the REAL input channels (weight.shape[1]): zero-padded input
        # channels (the MWT fusion conv's 54 -> 64) are not counted
        work = {'flops': 2.0 * N * Ho * Wo * Cout * k * k * Cin, 'bytes': (xc.numel() + y.numel() + wp.numel()) * 2}
        ctx.cap = L.current_cap()
        with L.launch_cap(ctx.cap):
            if bn_stats is not None:
                # BatchNorm statistics of y left by the epilogue (ewvit_bn_fwd_partials)
                shift, part, shift_out = bn_stats
                L.call('ewvit_conv2d_fwd_bn', L.ptr(xc), L.ptr(wp), L.ptr(b), L.ptr(y), N, H, W, Cx, Cout, k, stride,
                       gc, gs, L.ptr(shift), L.ptr(part), L.ptr(shift_out), L.stream(y), work=work)
            else:
                L.call('ewvit_conv2d_fwd', L.ptr(xc), L.ptr(wp), L.ptr(b), L.ptr(y), N, H, W, Cx, Cout, k, stride, gc,
                       gs, L.stream(y), work=work)
        ctx.save_for_backward(xc, weight, wpt)
        ctx.params = (weight, bias)          # gradient slots (ewvit.grads) are looked up on these
        ctx.cfg = (stride, levels, bias is not None, x.dtype)
        # bf16 MFMA product; an fp32 caller (no autocast) gets fp32 back
        return y if x.dtype == torch.bfloat16 else y.to(x.dtype).contiguous(memory_format=torch.channels_last)

    @staticmethod
    def backward(ctx, dy):
        with L.launch_cap(L.bwd_cap(ctx.cap)):
            return Conv2dFn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        xc, weight, wpt = ctx.saved_tensors
        stride, levels, has_bias, xdt = ctx.cfg
        NL, Cz, H, W = xc.shape
        N, Cx = NL // levels, Cz * levels
        gc, gs = (Cz, N * H * W * Cz) if levels > 1 else (0, 0)
        Cout, Cin, k = weight.shape[0], weight.shape[1], weight.shape[2]
        Ho, Wo = dy.shape[2], dy.shape[3]
        dyc = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = db = None
        link = ctx.link
        skip = link.grad if link is not None else None
        if link is not None:
            link.grad = None
        bl = ctx.bnlink
        ctx.bnlink = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(xc, memory_format=torch.channels_last)
            work = {'flops': 2.0 * N * Ho * Wo * Cin * k * k * Cout, 'bytes': (dyc.numel() + dx.numel() + wpt.numel()) * 2}
            lw = _bn_link_win(bl, xc, xdt, levels, N, H, W, Cx, Cout, k, stride, skip)
            lk = None if lw is not None else _bn_link_plan(bl, xc, xdt, levels, N, H, W, Cx, Cout, k, stride, skip)
            if lw is not None or lk is not None:
                # the backward-statistics epilogue also reads the BatchNorm's input (and the skip
                # gradient it adds): algorithmic bytes the kernel cannot avoid
                work['bytes'] += bl.x.numel() * bl.x.element_size() + (skip.numel() * 2 if skip is not None else 0)
            if lw is not None:
                # the windowed input gradient with the producing BatchNorm's per-block sums
                grows, rows = lw
                part = torch.empty(rows, 2 * Cx, dtype=torch.float32, device=xc.device)
                L.call('ewvit_conv2d_bwd_data_bn_win', L.ptr(dyc), L.ptr(wpt), L.ptr(dx), N, H, W, Cx, Cout, Cx, 0,
                       L.ptr(bl.x), L.ptr(bl.mean), L.ptr(bl.invstd), L.ptr(bl.gamma), L.ptr(bl.beta), bl.act, grows,
                       L.ptr(part), L.stream(dx), work=work)
                bl.fulfil(*bnmod.fold_bwd_partials(part, rows // bl.groups, bl.groups, Cx), dx)
            elif lk is not None:
                # dx (+ the skip gradient) and the producing BatchNorm's backward sums in one epilogue
                groups, grows, rows, Cg = lk
                sk = skip.to(torch.bfloat16).contiguous(memory_format=torch.channels_last) if skip is not None else None
                part = torch.empty(groups * rows, 2 * Cg, dtype=torch.float32, device=xc.device)
                nrc = ctypes.c_int(0)
                L.call('ewvit_conv2d_bwd_data_bn', L.ptr(dyc), L.ptr(wpt), L.ptr(dx), L.ptr(sk), N, H, W, Cx, Cout,
                       k, stride, gc, gs, L.ptr(bl.x), L.ptr(bl.mean), L.ptr(bl.invstd), L.ptr(bl.gamma),
                       L.ptr(bl.beta), bl.act, L.ptr(bl.rscale), grows, L.ptr(part), ctypes.byref(nrc), L.stream(dx),
                       work=work)
                bl.fulfil(*bnmod.fold_bwd_partials(part, nrc.value, groups, Cg), dx)
                skip = None
            elif skip is not None and L.load().ewvit_conv2d_bwd_data_add_ok(N, H, W, Cx, Cout, k, stride):
                # the residual block's skip gradient added in the dgrad epilogue
                sk = skip.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                L.call('ewvit_conv2d_bwd_data_add', L.ptr(dyc), L.ptr(wpt), L.ptr(dx), L.ptr(sk), N, H, W, Cx, Cout,
                       k, stride, L.stream(dx), work=work)
                skip = None
            else:
                L.call('ewvit_conv2d_bwd_data', L.ptr(dyc), L.ptr(wpt), L.ptr(dx), N, H, W, Cx, Cout, k, stride, gc,
                       gs, L.stream(dx), work=work)
            if xdt != torch.bfloat16:
                dx = dx.to(xdt)
            if skip is not None:
                dx = dx + skip.to(dx.dtype)
        want_b = has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            wparam, bparam = ctx.params
            dw, db = Conv2dFn._wgrad(ctx, xc, dyc, weight, wparam, bparam, want_b, N, H, W, Cx, Cout, Cin, k,
                                     stride, Ho, Wo, gc, gs)
        if dx is None and skip is not None:       # x needs no gradient through the conv, only the skip's
            dx = skip
        if dw is not None or db is not None:
            wparam, bparam = ctx.params
            dw, db = grads.give(wparam, dw, ctx.gen), grads.give(bparam, db, ctx.gen)
        return dx, dw, db, None, None, None

    @staticmethod
    def _wgrad(ctx, xc, dyc, weight, wparam, bparam, want_b, N, H, W, Cx, Cout, Cin, k, stride, Ho, Wo, gc, gs):
        """dW (and db) on the current stream."""
        wsb = L.load().ewvit_conv2d_bwd_weight_workspace(N, H, W, Cx, Cout, k, stride)
        ws = torch.empty(wsb // 4, dtype=torch.float32, device=xc.device)
        # dW in the parameter's own memory format — the data-parallel flat buffer's view
        # when the step provides one (ewvit.grads), so no copy or layout change follows
        dwf = grad_out(wparam, ctx.gen) if ctx.needs_input_grad[1] else torch.empty_like(weight, dtype=torch.float32)
        s_co, s_ci, s_kh, s_kw = dwf.stride()
        if s_kh != k * s_kw:
            dwf = torch.empty((Cout, Cin, k, k), dtype=torch.float32, device=xc.device)
            s_co, s_ci, s_kh, s_kw = dwf.stride()
        dbf = None
        if want_b:
            dbf = grad_out(bparam, ctx.gen)
            if dbf.dim() != 1 or not dbf.is_contiguous():
                dbf = torch.empty(Cout, dtype=torch.float32, device=xc.device)
        work = {'flops': 2.0 * N * Ho * Wo * Cout * k * k * Cin, 'bytes': (dyc.numel() + xc.numel()) * 2}
        if ctx.needs_input_grad[1] and dbf is None and grads.deferrable(wparam, dwf, ctx.gen) and _defer.available():
            # dW is read by nobody before the end of the backward (ewvit.grads.deferrable): the
            # split-K reduce rides in a later weight-gradient launch (ewvit.defer)
            _defer.mark(ws, dwf, xc.device)
        L.call('ewvit_conv2d_bwd_weight', L.ptr(xc), L.ptr(dyc), L.ptr(dwf), L.ptr(dbf), 0, N, H, W, Cx,
               Cout, k, stride, gc, gs, Cin, s_co, s_ci, s_kw, L.ptr(ws), L.stream(dwf), work=work)
        return (dwf if ctx.needs_input_grad[1] else None), dbf


def conv2d(x, weight, bias=None, stride=1, levels=1):
    """Conv2d(kernel 1|3, padding k//2, stride) — NCHW logical / channels-last bf16 output.
    levels > 1: x is level-major [levels*N, C, H, W], convolved as cat(x.chunk(levels), 1)."""
    return Conv2dFn.apply(x, weight, bias, int(stride), int(levels))


def bn_stat_rows(x, weight, stride=1, levels=1):
    """Rows per BatchNorm partial that `conv2d_bn_stats` leaves for this conv (the LDS-DMA
    kernel's m-tile), or 0 when the conv cannot produce them (then use conv2d + BN)."""
    NL, Cz, H, W = x.shape
    k = weight.shape[2]
    Cx = Cz * levels
    if (not x.is_cuda or Cx < weight.shape[1] or (levels > 1 and Cx != weight.shape[1]) or k not in (1, 3)
            or weight.shape[3] != k or weight.shape[0] % 8 or NL % levels or (levels > 1 and Cz % 64)):
        return 0
    return int(L.load().ewvit_conv2d_fwd_bn_rows(NL // levels, H, W, Cz * levels, weight.shape[0], k, int(stride)))


def conv2d_bn_stats(x, weight, bias, stride, shift, levels=1, groups=1, max_rows=256):
    """conv2d whose epilogue also leaves the BatchNorm partial statistics of its bf16
    output: returns (y, part [groups, nrc, 2*Cout], shifts [groups, Cout], nrc) for
    ewvit.bn.batch_norm_act(..., partials=(part, shifts, nrc)), or None when the shape
    is not supported.  `shift` (the BN running mean) centres the sums; `groups` equal
    batch slices get separate statistics (each must be whole output tiles); more than
    `max_rows` tile rows per group are folded by one extra launch."""
    rows = bn_stat_rows(x, weight, stride, levels)
    if rows <= 0:
        return None
    NL, _, H, W = x.shape
    N = NL // levels
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    M = N * Ho * Wo
    if M % groups or (groups > 1 and (M // groups) % rows):
        return None
    Cout = weight.shape[0]
    nrc = (M // groups + rows - 1) // rows
    part = torch.empty(groups * nrc, 2 * Cout, dtype=torch.float32, device=x.device)
    shifts = torch.empty(Cout, dtype=torch.float32, device=x.device)
    sh = shift.detach().float().contiguous() if shift is not None else None
    y = Conv2dFn.apply(x, weight, bias, int(stride), int(levels), (sh, part, shifts))
    if nrc > max_rows or groups > 1:
        nout = min(nrc, max_rows)
        part2 = torch.empty(groups, nout, 2 * Cout, dtype=torch.float32, device=x.device)
        shifts2 = torch.empty(groups, Cout, dtype=torch.float32, device=x.device)
        L.call('ewvit_bn_fold_partials', L.ptr(part), nrc, L.ptr(shifts), L.ptr(part2), nout, L.ptr(shifts2), Cout,
               groups, L.stream(y))
        part, shifts, nrc = part2, shifts2, nout
    return y, part, shifts, nrc


# BnReluConvFn's BatchNorm backward sums taken by the conv's windowed input-gradient epilogue
# (ewvit_conv2d_bwd_data_bn_win; False: ewvit_bn_bwd's own reduction pass, A/B and tests)
_BN_BWD_EPI = os.environ.get('EWVIT_BN_BWD_EPI', '1') != '0'


class BnReluConvFn(torch.autograd.Function):
    """conv3x3(relu(BatchNorm(z))) in training, the BatchNorm + ReLU applied inside the windowed
    conv's operand staging (ewvit_conv2d_fwd_bn_xf / ewvit_conv2d_bwd_weight_xf): the normalised
    map is never written.  z is the level-major producer output [levels*N, C, H, W] whose
    BatchNorm statistics (per level) its producer's epilogue summed (`zpart` = (part, shifts,
    nrc)); the conv reads the levels as channel groups (mwt.py:112's concatenation).  Forward:
    ewvit_bn_coef (the BN's finalisation: batch / running statistics, counter, scale and shift)
    + the transformed conv with the next BatchNorm's statistics (`ystats`).  Backward: the
    conv's input gradient (it does not read z) with the BatchNorm backward sums in its epilogue,
    the transformed weight gradient, then the BatchNorm + ReLU backward's dx pass on z.  With
    _BN_BWD_EPI off the BN backward runs its own reduction (ewvit_bn_bwd) — then the same
    kernels in the same order as BatchNormActFn followed by Conv2dFn, every result bit-identical
    to that pair; with it on the sums are the same values summed in another order."""

    @staticmethod
    def forward(ctx, z, weight, bias, gamma, beta, running_mean, running_var, momentum, eps, counter, levels, zpart,
                ystats):
        L.require_gpu(z, weight)
        ctx.cap = L.current_cap()
        with L.launch_cap(ctx.cap):
            return BnReluConvFn._forward(ctx, z, weight, bias, gamma, beta, running_mean, running_var, momentum, eps,
                                         counter, levels, zpart, ystats)

    @staticmethod
    def _forward(ctx, z, weight, bias, gamma, beta, running_mean, running_var, momentum, eps, counter, levels, zpart,
                 ystats):
        zc = z.contiguous(memory_format=torch.channels_last)
        NL, C, H, W = zc.shape
        N, Cx = NL // levels, C * levels
        Cout = weight.shape[0]
        dev = z.device
        part, shifts, nrc = zpart
        M = NL * H * W
        coef = torch.empty(levels, 2, C, dtype=torch.float32, device=dev)
        mean = torch.empty(levels, C, dtype=torch.float32, device=dev)
        invstd = torch.empty_like(mean)
        L.call('ewvit_bn_coef', M, C, L.ptr(gamma), L.ptr(beta), L.ptr(running_mean), L.ptr(running_var),
               float(momentum), float(eps), L.ptr(mean), L.ptr(invstd), L.ptr(counter), L.ptr(part), L.ptr(shifts),
               int(nrc), levels, L.ptr(coef), L.stream(zc))
        cached = _cached_pack(weight, Cx, True) if weight.dtype == torch.float32 else None
        if cached is None:
            wp, wpt = _pack(weight, Cx, True, True)
            if weight.dtype == torch.float32:
                _register(weight, Cx, True)
        else:
            wp, wpt = cached
        y = torch.empty((N, Cout, H, W), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        b = bias.detach().float().contiguous() if bias is not None else None
        shift, ypart, yshift = ystats
        gs = N * H * W * C
        L.call('ewvit_conv2d_fwd_bn_xf', L.ptr(zc), L.ptr(wp), L.ptr(b), L.ptr(y), N, H, W, Cx, Cout, C, gs,
               L.ptr(coef), L.ptr(shift), L.ptr(ypart), L.ptr(yshift), L.stream(y),
               work={'flops': 2.0 * N * H * W * Cout * 9 * Cx, 'bytes': (zc.numel() + y.numel() + wp.numel()) * 2})
        ctx.save_for_backward(zc, weight, wpt, coef, gamma, beta, mean, invstd)
        ctx.gen = grads.note_use(weight)
        for t in (bias, gamma, beta):
            grads.note_use(t)
        ctx.params = (weight, bias, gamma, beta)
        ctx.cfg = (levels, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        with L.launch_cap(L.bwd_cap(ctx.cap)):
            return BnReluConvFn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        zc, weight, wpt, coef, gamma, beta, mean, invstd = ctx.saved_tensors
        levels, has_bias = ctx.cfg
        NL, C, H, W = zc.shape
        N, Cx = NL // levels, C * levels
        Cout = weight.shape[0]
        gs = N * H * W * C
        dev = zc.device
        dyc = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        # d relu(bn(z)) — the input gradient of the conv, in z's level-major layout — and the BN
        # backward's per-block sums of g = da * relu'(.) and g * xhat
        da = torch.empty_like(zc, memory_format=torch.channels_last)
        work = {'flops': 2.0 * N * H * W * Cx * 9 * Cout, 'bytes': (dyc.numel() + da.numel() + wpt.numel()) * 2}
        rows = int(L.load().ewvit_conv2d_bwd_bn_win_rows(N, H, W, Cx, Cout, 3, 1, C, gs, 0)) \
            if _BN_BWD_EPI and L.has('ewvit_conv2d_bwd_bn_win_rows') else 0
        bpart = None
        if rows > 0:
            work['bytes'] += zc.numel() * 2        # the BST epilogue reads the BatchNorm input z
            bpart = torch.empty(levels * rows, 2 * C, dtype=torch.float32, device=dev)
            L.call('ewvit_conv2d_bwd_data_bn_win', L.ptr(dyc), L.ptr(wpt), L.ptr(da), N, H, W, Cx, Cout, C, gs,
                   L.ptr(zc), L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), 1, 0, L.ptr(bpart), L.stream(da),
                   work=work)
        else:
            L.call('ewvit_conv2d_bwd_data', L.ptr(dyc), L.ptr(wpt), L.ptr(da), N, H, W, Cx, Cout, 3, 1, C, gs,
                   L.stream(da), work=work)
        wparam, bparam, gparam, beparam = ctx.params
        dwf = grad_out(wparam, ctx.gen)
        s_co, s_ci, s_kh, s_kw = dwf.stride()
        if s_kh != 3 * s_kw:
            dwf = torch.empty((Cout, Cx, 3, 3), dtype=torch.float32, device=dev)
            s_co, s_ci, s_kh, s_kw = dwf.stride()
        dbf = None
        if has_bias:
            dbf = grad_out(bparam, ctx.gen)
            if dbf.dim() != 1 or not dbf.is_contiguous():
                dbf = torch.empty(Cout, dtype=torch.float32, device=dev)
        ws = torch.empty(L.load().ewvit_conv2d_bwd_weight_workspace(N, H, W, Cx, Cout, 3, 1) // 4, dtype=torch.float32,
                         device=dev)
        L.call('ewvit_conv2d_bwd_weight_xf', L.ptr(zc), L.ptr(dyc), L.ptr(dwf), L.ptr(dbf), 0, N, H, W, Cx, Cout, C, gs,
               L.ptr(coef), Cx, s_co, s_ci, s_kw, L.ptr(ws), L.stream(dwf),
               work={'flops': 2.0 * N * H * W * Cout * 9 * Cx, 'bytes': (dyc.numel() + zc.numel()) * 2})
        # BatchNorm + ReLU backward on z (per level)
        M = NL * H * W
        dz = torch.empty_like(zc)
        dg = bnmod._affine_grad(gparam, ctx.gen, C, dev)
        db2 = bnmod._affine_grad(beparam, ctx.gen, C, dev)
        if bpart is not None:
            p2, n2 = bnmod.fold_bwd_partials(bpart, rows, levels, C)
            L.call('ewvit_bn_bwd_partials', L.ptr(da), L.ptr(zc), L.ptr(dz), L.dt(zc), M, C, L.ptr(gamma), L.ptr(beta),
                   L.ptr(mean), L.ptr(invstd), 1, L.ptr(dg), L.ptr(db2), None, 1, L.ptr(p2), n2, levels, L.stream(dz),
                   work={'bytes': 3 * zc.numel() * zc.element_size()})
        else:
            bws = torch.empty(L.load().ewvit_bn_workspace(M, C, levels) // 4, dtype=torch.float32, device=dev)
            L.call('ewvit_bn_bwd', L.ptr(da), L.ptr(zc), L.ptr(dz), L.dt(zc), M, C, L.ptr(gamma), L.ptr(beta),
                   L.ptr(mean), L.ptr(invstd), 1, L.ptr(dg), L.ptr(db2), 0, levels, L.ptr(bws), L.stream(dz),
                   work={'bytes': 5 * zc.numel() * zc.element_size()})
        g = ctx.gen
        return (dz, grads.give(wparam, dwf, g), grads.give(bparam, dbf, g) if has_bias else None,
                grads.give(gparam, dg, g), grads.give(beparam, db2, g), *(None,) * 8)


def bn_relu_ok(z, weight, levels):
    """True when bn_relu_conv2d_bn_stats takes this (producer output z, 3x3 conv weight) pair."""
    if not (z.is_cuda and z.dim() == 4 and z.dtype == torch.bfloat16 and weight.dim() == 4
            and tuple(weight.shape[2:]) == (3, 3) and weight.dtype == torch.float32 and z.shape[0] % levels == 0
            and weight.shape[1] == z.shape[1] * levels):
        return False
    NL, C, H, W = z.shape
    N = NL // levels
    return bool(L.load().ewvit_conv2d_xf_ok(N, H, W, C * levels, weight.shape[0], 3, 1, C, N * H * W * C))


def bn_relu_conv2d_bn_stats(z, zpart, bn, weight, bias, shift, levels, max_rows=256):
    """conv3x3(relu(bn(z)), weight, bias) for a training BatchNorm module `bn` whose batch
    statistics (one group per level of the level-major z) its producer summed (`zpart`), with
    the conv's own output statistics for the next BatchNorm: (y, part, shifts, nrc) as
    conv2d_bn_stats.  See BnReluConvFn."""
    NL, C, H, W = z.shape
    N = NL // levels
    Cout = weight.shape[0]
    rows = 256
    nrc = (N * H * W + rows - 1) // rows
    part = torch.empty(nrc, 2 * Cout, dtype=torch.float32, device=z.device)
    shifts = torch.empty(Cout, dtype=torch.float32, device=z.device)
    sh = shift.detach().float().contiguous() if shift is not None else None
    counter = bn.num_batches_tracked if bn.track_running_stats else None
    y = BnReluConvFn.apply(z, weight, bias, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                           counter, int(levels), zpart, (sh, part, shifts))
    if nrc > max_rows:
        part2 = torch.empty(1, max_rows, 2 * Cout, dtype=torch.float32, device=z.device)
        shifts2 = torch.empty(1, Cout, dtype=torch.float32, device=z.device)
        L.call('ewvit_bn_fold_partials', L.ptr(part), nrc, L.ptr(shifts), L.ptr(part2), max_rows, L.ptr(shifts2), Cout,
               1, L.stream(y))
        part, shifts, nrc = part2, shifts2, max_rows
    return y, part, shifts, nrc


def stem_ok(x, weight, bias, stride):
    """The frozen backbone stem's shape class (ewvit_conv2d_stem_fwd): 3x3, pad 1, stride
    1|2, Cin 1..4, Cout 8/16/24/32, f32 / bf16 input, no gradient needed anywhere."""
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16) and weight.dim() == 4
            and tuple(weight.shape[2:]) == (3, 3) and 1 <= weight.shape[1] <= 4 and x.shape[1] == weight.shape[1]
            and weight.shape[0] in (8, 16, 24, 32) and weight.dtype == torch.float32 and stride in (1, 2)
            and not (torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad
                                                  or (bias is not None and bias.requires_grad))))


_stem_bufs = {}       # id(weight) -> (weakref(weight), padded buffer)


def _stem_weight(weight, bias):
    """The weight as the stem kernel reads it: tap-major [Cin*9][Cout] fp32, the bias as
    one more row (if any), then 64 padding floats (its scalar loads take 64 bytes at a
    time).  The buffer persists per parameter; the permuting copy into it is one small
    launch per call (two with a bias), so a graph-replayed step always reads the
    parameters' current values."""
    Cout, n = weight.shape[0], weight.numel()
    size = n + (Cout if bias is not None else 0) + 64
    e = _stem_bufs.get(id(weight))
    buf = e[1] if e is not None and e[0]() is weight else None
    if buf is None or buf.device != weight.device or buf.numel() != size:
        buf = torch.zeros(size, dtype=torch.float32, device=weight.device)
        _stem_bufs[id(weight)] = (weakref.ref(weight), buf)
    buf[:n].view(n // Cout, Cout).copy_(weight.detach().permute(1, 2, 3, 0).reshape(n // Cout, Cout))
    if bias is not None:
        buf[n:n + Cout].copy_(bias.detach())
    return buf


def stem_conv2d(x, weight, bias, stride, shift=None, stats=False, max_rows=256):
    """Forward-only direct conv of the backbone stem (csrc/stem.hip; reference
    sfe.py:111-119 freezes it): y bf16 channels-last.  stats=True also returns the
    BatchNorm partial statistics of y centred on `shift` — (y, part, shifts, nrc) as
    conv2d_bn_stats — folded to <= max_rows rows."""
    assert stem_ok(x, weight, bias, stride), 'stem_conv2d: unsupported shape or a gradient is required'
    N, Cin, H, W = x.shape
    Cout = weight.shape[0]
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    part = shifts = sh = None
    nrc = 0
    if stats:
        nrc = int(L.load().ewvit_conv2d_stem_parts(N, H, W, int(stride)))
        part = torch.empty(nrc, 2 * Cout, dtype=torch.float32, device=x.device)
        shifts = torch.empty(Cout, dtype=torch.float32, device=x.device)
        sh = shift.detach().float().contiguous() if shift is not None else None
    w = _stem_weight(weight, bias)
    L.call('ewvit_conv2d_stem_fwd', L.ptr(x), L.dt(x), N, Cin, H, W, *x.stride(), L.ptr(w), int(bias is not None),
           L.ptr(y), Cout, int(stride), L.ptr(sh), L.ptr(part), L.ptr(shifts), L.stream(x))
    if not stats:
        return y
    if nrc > max_rows:
        part2 = torch.empty(1, max_rows, 2 * Cout, dtype=torch.float32, device=x.device)
        shifts2 = torch.empty(1, Cout, dtype=torch.float32, device=x.device)
        L.call('ewvit_bn_fold_partials', L.ptr(part), nrc, L.ptr(shifts), L.ptr(part2), max_rows, L.ptr(shifts2),
               Cout, 1, L.stream(y))
        part, shifts, nrc = part2, shifts2, max_rows
    return y, part, shifts, nrc


def conv3x3(x, weight, bias=None, stride=1):
    """Conv2d(kernel 3, padding 1, stride)."""
    return Conv2dFn.apply(x, weight, bias, int(stride), 1)
