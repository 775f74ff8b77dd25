"""The DAMA frame head on csrc/head.hip — everything of DAMA._process_frame after its two
branches (reference network/dama.py:143-169): the 2-layer bidirectional cross-attention, the
fusion gate (centre-tap conv + BatchNorm + ReLU), the gate net and the 3-way weighted sum.

Forward: one workgroup per 16 frames (the attention blocks, fusion conv and gate input layer,
LDS-resident) + one workgroup for the frame-coupled tail (BatchNorm over the frames, gate
softmax, weighted sum); backward: the tail, the frame groups in reverse, and one grid for the
parameter gradients.  The module-by-module path (network/dama.py) issues ~90 small launches
for the same work; it stays for hooked / patched modules and shapes outside this kernel's
class (dim 128, 4 heads of 32, depth 2, <= 64 frames).  With fp8 token GEMMs (mx=True) the
attention blocks' GEMMs run on MXFP8 operands (a second weight pack, ewvit_head_pack_bytes_mx).
"""
import ctypes

import torch

from . import _lib as L
from . import grads
from .grads import grad_out

_vp, _i64, _f32, _u64, _i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64, ctypes.c_int


class _CA(ctypes.Structure):
    _fields_ = [('ln_w', _vp), ('ln_b', _vp), ('wq', _vp), ('wkv', _vp), ('wo', _vp), ('bo', _vp)]


class _Params(ctypes.Structure):
    """include/ewvit.h ewvit_head_params."""
    _fields_ = [('ca', _CA * 4), ('wfg', _vp), ('fg_so', _i64), ('fg_si', _i64), ('fg_tap', _i64), ('bfg', _vp),
                ('bn_w', _vp), ('bn_b', _vp), ('bn_rm', _vp), ('bn_rv', _vp), ('bn_nbt', _vp), ('bn_mom', _f32),
                ('bn_eps', _f32), ('g1w', _vp), ('g1b', _vp), ('g2w', _vp), ('g2b', _vp), ('p_ca', _f32),
                ('p_gate', _f32), ('seed', _u64), ('seed_off', _vp), ('training', _i32), ('ln_eps', _f32),
                ('packed', _vp), ('packed_mx', _vp)]


class HeadCfg:
    """The non-tensor state of one call: BatchNorm buffers and hyper-parameters, dropout."""

    def __init__(self, bn, ln_eps, p_ca, p_gate, training, seed, mx=False):
        self.bn, self.ln_eps, self.p_ca, self.p_gate, self.training, self.seed = bn, ln_eps, p_ca, p_gate, training, seed
        self.mx = bool(mx)


def _params(cfg, ts, dev, packed=None, packed_mx=None):
    p = _Params()
    p.packed = packed
    p.packed_mx = packed_mx
    for i in range(4):
        lw, lb, wq, wkv, wo, bo = ts[6 * i:6 * i + 6]
        p.ca[i] = _CA(lw.data_ptr(), lb.data_ptr(), wq.data_ptr(), wkv.data_ptr(), wo.data_ptr(), bo.data_ptr())
    wfg, bfg, bnw, bnb, g1w, g1b, g2w, g2b = ts[24:32]
    p.wfg = wfg.data_ptr()
    p.fg_so, p.fg_si = wfg.stride(0), wfg.stride(1)
    p.fg_tap = wfg.stride(3)
    p.bfg = bfg.data_ptr()
    bn = cfg.bn
    p.bn_w, p.bn_b = bnw.data_ptr(), bnb.data_ptr()
    p.bn_rm, p.bn_rv = bn.running_mean.data_ptr(), bn.running_var.data_ptr()
    p.bn_nbt = bn.num_batches_tracked.data_ptr() if (cfg.training and bn.num_batches_tracked is not None) else None
    p.bn_mom, p.bn_eps = float(bn.momentum), float(bn.eps)
    p.g1w, p.g1b, p.g2w, p.g2b = g1w.data_ptr(), g1b.data_ptr(), g2w.data_ptr(), g2b.data_ptr()
    p.p_ca, p.p_gate = (cfg.p_ca, cfg.p_gate) if cfg.training else (0.0, 0.0)
    p.seed = cfg.seed
    p.seed_off = L.rng_offset(dev).data_ptr()
    p.training = int(cfg.training)
    p.ln_eps = float(cfg.ln_eps)
    return p


class DamaHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, s0, f0, *ts):
        L.require_gpu(s0, f0, *ts)
        N = s0.shape[0]
        s0c, f0c = s0.float().contiguous(), f0.float().contiguous()
        ts = tuple(t if t.dtype == torch.float32 else t.float() for t in ts)
        dev = s0.device
        ws = torch.empty(int(L.load().ewvit_head_workspace()) // 4, dtype=torch.float32, device=dev)
        pk = torch.empty(int(L.load().ewvit_head_pack_bytes()), dtype=torch.uint8, device=dev)
        pkm = torch.empty(int(L.load().ewvit_head_pack_bytes_mx()), dtype=torch.uint8, device=dev) if cfg.mx else None
        fused = torch.empty(N, 128, dtype=torch.float32, device=dev)
        so, fo = torch.empty_like(fused), torch.empty_like(fused)
        p = _params(cfg, ts, dev, pk.data_ptr(), pkm.data_ptr() if pkm is not None else None)
        ctx.gen = grads.note_use(ts[0])
        for t in ts[1:]:
            grads.note_use(t)
        L.call('ewvit_head_fwd', ctypes.addressof(p), L.ptr(s0c), L.ptr(f0c), N, L.ptr(ws), L.ptr(fused), L.ptr(so),
               L.ptr(fo), L.stream(fused), work={'flops': 2.0 * N * 128 * (4 * (128 + 512 + 128) + 256 + 64),
                                                 'bytes': 4.0 * sum(t.numel() for t in ts)})
        ctx.cfg, ctx.N, ctx.ts = cfg, N, ts
        ctx.save_for_backward(ws, pk, *(() if pkm is None else (pkm,)))
        return fused, so, fo

    @staticmethod
    def backward(ctx, g_fused, g_s, g_f):
        ws, pk, *pkm = ctx.saved_tensors
        cfg, N, ts = ctx.cfg, ctx.N, ctx.ts
        dev = ws.device

        def g32(g):
            return torch.zeros(N, 128, dtype=torch.float32, device=dev) if g is None else g.float().contiguous()
        gF, gS, gFr = g32(g_fused), g32(g_s), g32(g_f)
        ds0, df0 = torch.empty(N, 128, dtype=torch.float32, device=dev), torch.empty(N, 128, dtype=torch.float32,
                                                                                         device=dev)
        outs = []
        for k, t in enumerate(ts):
            # the kernel writes every parameter's gradient; a frozen one gets a scratch tensor
            g = grad_out(t, ctx.gen) if ctx.needs_input_grad[3 + k] else torch.empty_like(t)
            if k == 24 and g.stride() != t.stride():
                g = torch.empty_like(t)
            outs.append(g)
        p = _params(cfg, ts, dev, pk.data_ptr(), pkm[0].data_ptr() if pkm else None)
        arr = ctypes.c_void_p * 4

        def col(j):
            return arr(*[outs[6 * i + j].data_ptr() for i in range(4)])
        wfg = outs[24]
        L.call('ewvit_head_bwd', ctypes.addressof(p), L.ptr(ws), N, L.ptr(gF), L.ptr(gS), L.ptr(gFr), L.ptr(ds0),
               L.ptr(df0), col(2), col(3), col(4), col(5), col(0), col(1), L.ptr(wfg), wfg.stride(0), wfg.stride(1),
               wfg.stride(3), L.ptr(outs[25]), L.ptr(outs[26]), L.ptr(outs[27]), L.ptr(outs[28]), L.ptr(outs[29]),
               L.ptr(outs[30]), L.ptr(outs[31]), L.stream(ds0),
               work={'flops': 4.0 * N * 128 * (4 * (128 + 512 + 128) + 256 + 64), 'bytes': 8.0 * sum(t.numel() for t in ts)})
        return (None, ds0, df0, *[grads.give(t, g, ctx.gen) if ctx.needs_input_grad[3 + k] else None
                                  for k, (t, g) in enumerate(zip(ts, outs))])


def params_of(dama):
    """The 32 parameter tensors of DAMA's head, in the kernel's order."""
    ts = []
    for layer in dama.cross_att.layers:
        for norm, att in ((layer[0], layer[1]), (layer[2], layer[3])):
            ts += [norm.weight, norm.bias, att.to_q.weight, att.to_kv.weight, att.to_out[0].weight, att.to_out[0].bias]
    # kernel order: layer 0 s, layer 0 f, layer 1 s, layer 1 f — as built above
    fg = dama.fusion_gate
    gn = dama.gate_net
    ts += [fg[0].weight, fg[0].bias, fg[1].weight, fg[1].bias, gn[2].weight, gn[2].bias, gn[5].weight, gn[5].bias]
    return ts


def dama_head(dama, s0, f0, seed, mx=False):
    """(fused, space, freq) per frame for s0, f0 [N, 128]: DamaHeadFn with DAMA's parameters
    (mx: the attention blocks' GEMMs on MXFP8 operands)."""
    bn = dama.fusion_gate[1]
    att = dama.cross_att.layers[0][1]
    cfg = HeadCfg(bn, dama.cross_att.layers[0][0].eps, att.to_out[1].p, dama.gate_net[4].p, dama.training, seed, mx)
    return DamaHeadFn.apply(cfg, s0, f0, *params_of(dama))
