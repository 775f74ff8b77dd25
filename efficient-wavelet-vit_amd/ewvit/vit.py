"""One pre-norm ViT encoder layer of the spatial branch on csrc/vit.hip (reference
network/sfe.py:72-85: x = Attention(LN(x)) + x; x = FeedForward(LN(x)) + x).

At the hot path's shape — dim 512, 8 heads of 64, mlp 2048, 2 tokens per frame, <= 64 frames —
the layer is 4 forward and 5 backward launches instead of the module path's 11 and ~25
(LayerNorm, to_qkv, attention, to_out, LayerNorm, two Linears, their split-K reduces, the
activation / dropout backward and column sums): every GEMM there is 128 rows against a fp32
weight, so the layer is launch latency, not bytes or flops.  Roundings are the module path's
(bf16 MFMA operands where ewvit_gemm rounds them, the bf16 attention output and dh), and the
to_out dropout draws the same host seed and device counter, so the two paths agree to fp32
summation order.  `network.sfe.Transformer` takes this path when the layer is in its shape
class and nothing is hooked or patched (EWVIT_VIT_FUSED=0 keeps the module path).
"""
import ctypes
import os

import torch

from . import _lib as L
from . import grads
from .grads import grad_out

_vp, _f32, _u64 = ctypes.c_void_p, ctypes.c_float, ctypes.c_uint64


class _Params(ctypes.Structure):
    """include/ewvit.h ewvit_vit_layer."""
    _fields_ = [('ln1_w', _vp), ('ln1_b', _vp), ('wqkv', _vp), ('wo', _vp), ('bo', _vp), ('ln2_w', _vp),
                ('ln2_b', _vp), ('w1', _vp), ('b1', _vp), ('w2', _vp), ('b2', _vp), ('ln_eps', _f32),
                ('drop_p', _f32), ('seed', _u64), ('seed_off', _vp), ('packed', _vp), ('mx', ctypes.c_int)]


class _Grads(ctypes.Structure):
    """include/ewvit.h ewvit_vit_grads."""
    _fields_ = [(n, _vp) for n in ('ln1_w', 'ln1_b', 'wqkv', 'wo', 'bo', 'ln2_w', 'ln2_b', 'w1', 'b1', 'w2', 'b2')]


_WS = {}


def _ws_bytes(which):
    if which not in _WS:
        _WS[which] = int(L.load().ewvit_vit_layer_workspace(which))
    return _WS[which]


def enabled():
    return os.environ.get('EWVIT_VIT_FUSED', '1') != '0'


def params_of(attn, ff):
    """The 11 parameter tensors of one layer (PreNorm(Attention), PreNorm(FeedForward)) in the
    kernel's order."""
    a, f = attn.fn, ff.fn
    return [attn.norm.weight, attn.norm.bias, a.to_qkv.weight, a.to_out[0].weight, a.to_out[0].bias,
            ff.norm.weight, ff.norm.bias, f.net[0].weight, f.net[0].bias, f.net[3].weight, f.net[3].bias]


def _params(ts, eps, drop_p, seed, dev, packed=None, mx=False):
    p = _Params(*[t.data_ptr() for t in ts])
    p.ln_eps, p.drop_p, p.seed = float(eps), float(drop_p), int(seed)
    p.seed_off = L.rng_offset(dev).data_ptr() if drop_p > 0 else None
    p.packed = packed
    p.mx = int(bool(mx))
    return p


PACK_MAX = 8     # EWVIT_VIT_PACK_MAX


def pack(layers, mx=False):
    """The GEMM operands of the given (attn, ff) layers — to_qkv, to_out, Linear1, Linear2,
    each in its own layout and transposed — packed by one launch once per forward: bf16
    (ewvit_vit_pack), or MXFP8 for fp8 token GEMMs (mx=True, ewvit_vit_pack_mx: e4m3 with one
    E8M0 scale per 32 elements along each image's K).  Returns the buffer (one block of
    ewvit_vit_layer_workspace(2 | 3) bytes per layer)."""
    assert 1 <= len(layers) <= PACK_MAX
    ts0 = params_of(*layers[0])
    dev = ts0[0].device
    blk = _ws_bytes(3 if mx else 2)
    buf = torch.empty(len(layers) * blk, dtype=torch.uint8, device=dev)
    arr = (_Params * len(layers))()
    for i, (attn, ff) in enumerate(layers):
        arr[i] = _params(params_of(attn, ff), 0.0, 0.0, 0, dev)
    nw = sum(t.numel() for t in params_of(*layers[0])[2:] if t.dim() == 2) * len(layers)
    L.call('ewvit_vit_pack_mx' if mx else 'ewvit_vit_pack', ctypes.addressof(arr), len(layers), L.ptr(buf),
           L.stream(buf), work={'bytes': 4.0 * nw + len(layers) * blk})
    return buf


class ViTLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, x0, *ts):
        L.require_gpu(x0, *ts)
        eps, drop_p, seed, buf, idx, mx = cfg
        B = x0.shape[0]
        R = 2 * B
        x0c = x0.float().contiguous()
        dev = x0.device
        saved = torch.empty(_ws_bytes(0), dtype=torch.uint8, device=dev)
        x2 = torch.empty_like(x0c)
        pk = buf.data_ptr() + idx * _ws_bytes(3 if mx else 2)
        p = _params(ts, eps, drop_p, seed, dev, pk, mx)
        ctx.gen = grads.note_use(ts[0])
        for t in ts[1:]:
            grads.note_use(t)
        L.call('ewvit_vit_layer_fwd', ctypes.addressof(p), R, L.ptr(x0c), L.ptr(saved), L.ptr(x2), L.stream(x2),
               work={'flops': 2.0 * R * 512 * (1536 + 512 + 2 * 2048), 'bytes': 4.0 * sum(t.numel() for t in ts)})
        ctx.cfg, ctx.R, ctx.ts, ctx.pk = cfg, R, ts, pk
        ctx.save_for_backward(x0c, saved)
        return x2

    @staticmethod
    def backward(ctx, g):
        x0c, saved = ctx.saved_tensors
        eps, drop_p, seed, buf, idx, mx = ctx.cfg
        ts, R = ctx.ts, ctx.R
        dev = x0c.device
        gc = g.float().contiguous()
        scratch = torch.empty(_ws_bytes(1), dtype=torch.uint8, device=dev)
        dx0 = torch.empty_like(x0c)
        outs = []
        for k, t in enumerate(ts):
            # the kernels write every parameter gradient; a frozen one gets a scratch tensor
            o = grad_out(t, ctx.gen) if ctx.needs_input_grad[2 + k] else torch.empty_like(t)
            outs.append(o if o.is_contiguous() else torch.empty_like(t, memory_format=torch.contiguous_format))
        p = _params(ts, eps, drop_p, seed, dev, ctx.pk, mx)
        G = _Grads(*[o.data_ptr() for o in outs])
        L.call('ewvit_vit_layer_bwd', ctypes.addressof(p), R, L.ptr(x0c), L.ptr(saved), L.ptr(gc), L.ptr(scratch),
               L.ptr(dx0), ctypes.addressof(G), L.stream(dx0),
               work={'flops': 4.0 * R * 512 * (1536 + 512 + 2 * 2048), 'bytes': 8.0 * sum(t.numel() for t in ts)})
        return (None, dx0.reshape(g.shape), *[grads.give(t, o, ctx.gen) if ctx.needs_input_grad[2 + k] else None
                                              for k, (t, o) in enumerate(zip(ts, outs))])


def vit_layer(attn, ff, x, training, packed, idx, mx=False):
    """x [B, 2, 512] -> the layer's output [B, 2, 512] f32 (ViTLayerFn with the layer's
    parameters and block `idx` of `packed` (ewvit.vit.pack, MXFP8 GEMMs when mx); the to_out
    dropout draws its host seed as the module path's Linear does)."""
    from .ops import _seed
    drop = attn.fn.to_out[1].p if training else 0.0
    cfg = (attn.norm.eps, float(drop), _seed() if drop > 0 else 0, packed, int(idx), bool(mx))
    return ViTLayerFn.apply(cfg, x, *params_of(attn, ff))


class EmbedFn(torch.autograd.Function):
    """tok = Dropout(cat(cls, y) + pos_embedding[0:B]) for one patch per frame (sfe.py:155-160):
    one launch each way instead of cat / add / dropout and their backward (slice, sums)."""

    @staticmethod
    def forward(ctx, drop_p, seed, y, cls, pos):
        L.require_gpu(y, cls, pos)
        B = y.shape[0]
        yc = y.float().reshape(B, 512).contiguous()
        tok = torch.empty(B, 2, 512, dtype=torch.float32, device=y.device)
        off = L.rng_offset(y.device) if drop_p > 0 else None
        ctx.gen = grads.note_use(cls)
        grads.note_use(pos)
        L.call('ewvit_vit_embed_fwd', L.ptr(yc), L.ptr(cls), L.ptr(pos), B, pos.shape[0], float(drop_p), int(seed), L.ptr(off),
               L.ptr(tok), L.stream(tok))
        ctx.cfg = (float(drop_p), int(seed), B, y.shape)
        ctx.params = (cls, pos)
        return tok

    @staticmethod
    def backward(ctx, g):
        drop_p, seed, B, yshape = ctx.cfg
        cls, pos = ctx.params
        gc = g.float().contiguous()
        dy = torch.empty(B, 512, dtype=torch.float32, device=g.device)
        dcls = grad_out(cls, ctx.gen) if ctx.needs_input_grad[3] else torch.empty_like(cls)
        dpos = grad_out(pos, ctx.gen) if ctx.needs_input_grad[4] else torch.empty_like(pos)
        off = L.rng_offset(g.device) if drop_p > 0 else None
        L.call('ewvit_vit_embed_bwd', L.ptr(gc), B, pos.shape[0], drop_p, seed, L.ptr(off), L.ptr(dy), L.ptr(dcls),
               L.ptr(dpos), L.stream(dy))
        return (None, None, dy.reshape(yshape), grads.give(cls, dcls, ctx.gen) if ctx.needs_input_grad[3] else None,
                grads.give(pos, dpos, ctx.gen) if ctx.needs_input_grad[4] else None)


def embed(y, cls, pos, drop_p):
    from .ops import _seed
    return EmbedFn.apply(float(drop_p), _seed() if drop_p > 0 else 0, y, cls, pos)
