"""DAMA — frequency<->spatial fusion (drop-in for reference network/dama.py:15-206).

Hot path on MI355X: the bidirectional cross-attention (1 query x 2 keys per
frame, kv_include_self) runs on ewvit kernels — LayerNorm, to_q / to_kv MFMA
GEMMs, the short-sequence attention and to_out with dropout + residual fused
into its epilogue.  ``fusion_gate``'s 3x3 conv sees a 1x1 map with zero padding
(dama.py:124-128 on the [N, 2D, 1, 1] concat), so only its centre tap is live:
it runs as one GEMM on W[:, :, 1, 1] (exactly the conv's value and gradients).
The frame-chunk loop and the per-video means keep the reference's semantics
(pos_embedding indexed by chunk position, BatchNorm statistics per chunk).
"""
import os

import torch
from torch import nn
from torch.nn import functional as F

import ewvit
from ewvit import probe

from . import bf16_compute, load_config
from .mwt import MWT
from .sfe import EfficientViT, LayerNorm, Linear, _fp8, _hooked


_SIDE = {}


# A/B of the capture order: the MWT forward recorded before the SFE forward
_MWT_FIRST = os.environ.get('EWVIT_MWT_FIRST', '0') == '1'


def _side_stream(device, main):
    """The MWT branch's stream, one per (device, main stream): replicas driven from several
    threads on their own streams (nn.DataParallel) never share one."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, main.cuda_stream)
    st = _SIDE.get(key)
    if st is None:
        st = _SIDE[key] = torch.cuda.Stream(device=torch.device('cuda', idx))
    return st


def _branch_streams():
    """The MWT branch runs on a second stream beside the backbone (EWVIT_BRANCH_STREAMS=0:
    one stream).  Uncapped, the MWT's big convs and BatchNorm passes take every CU and the
    two streams gain ~1 %; with their grids capped (_mwt_grid_cap) the backbone's
    latency-bound kernels keep most CUs: 2754 -> 2952 frames/s (tools/cap_ab.sh)."""
    return os.environ.get('EWVIT_BRANCH_STREAMS', '1') == '1'


MWT_GRID_CAP = 128          # measured at world 1; the same at world > 1 (see _mwt_grid_cap)


def _mwt_grid_cap(world=None):
    """Workgroups per big-grid MWT launch (LDS-DMA convs, BatchNorm passes) while the MWT
    shares the GPU with the backbone (EWVIT_MWT_GRID_CAP, 0 = uncapped): the MWT walks its
    tiles / rows on 128 of the 256 CUs (16 per XCD) and the backbone's latency-bound kernels
    keep the rest.  After the deferred weight-gradient reductions shortened the backbone's
    backward (round 6, config 2, same box, interleaved rounds, profiles/r06/s2/ab/cap_*.log):
    80 3480-3482, 96 3884-3894, 112 3868-3879, **128 3902-3917** frames/s.  With the tap-split
    windowed weight gradient (8 waves per workgroup) the MWT
    keeps pace on fewer CUs (config 2, same box, 2 rounds each, profiles/r05/ab/cap_sweep_ts.log):
    80 3502-3508, **96 3645-3654**, 104 3603-3606, 112 3604-3608, 128 3614-3621, 160 3539-3545
    frames/s.  Before it (round 5's first windowed kernels, profiles/r05/ab/cap_sweep*.log): 64
    2750, 96 3546, 112 3541, 120 3572, 128 3573-3586, 136 3507, 160 3519, 192 3464 (round 4's
    kernels: 160 best, 2952 against 2919 at 144).

    Data parallel (reference train.py:249-251 on N GPUs) uses the SAME cap: the bucket
    all-reduces' RCCL kernels (one workgroup per RCCL channel) run during the backward on the
    128 CUs the cap leaves outside the MWT, beside the backbone's backward, whose 7^2-28^2
    launches fill 50-800 workgroups and leave CU slots between them.  Taking a
    reserve off the MWT instead would only move the MWT off its measured balance point (cap 96:
    -0.6 %, cap 80: -11 % at world 1).  No multi-GPU node was available to sweep the world > 1 budget, so the
    argument is kept for that sweep: EWVIT_MWT_GRID_CAP overrides the cap at every world size."""
    env = os.environ.get('EWVIT_MWT_GRID_CAP')
    if env is not None:
        return int(env)
    if world is None:
        import torch.distributed as dist
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    return MWT_GRID_CAP


class CrossAttention(nn.Module):                                           # dama.py:15-53
    def __init__(self, dim, heads=8, dim_head=64, dropout=0.):
        super().__init__()
        inner_dim = dim_head * heads
        project_out = not (heads == 1 and dim_head == dim)
        self.heads = heads
        self.dim_head = dim_head
        self.scale = dim_head ** -0.5
        self.attend = nn.Softmax(dim=-1)
        self.to_q = Linear(dim, inner_dim, bias=False)
        self.to_kv = Linear(dim, inner_dim * 2, bias=False)
        self.to_out = nn.Sequential(Linear(inner_dim, dim), nn.Dropout(dropout)) if project_out else nn.Identity()

    def forward(self, x, context=None, kv_include_self=False):
        return self.forward_residual(x, context, kv_include_self, None)

    def forward_residual(self, x, context=None, kv_include_self=False, resid=None):
        context = context if context is not None else x
        if kv_include_self:
            context = torch.cat((x.float(), context.float()), dim=1)
        q = ewvit.linear(x, self.to_q.weight, None, out_dtype=torch.bfloat16, fp8=_fp8(self.to_q))
        kv = ewvit.linear(context, self.to_kv.weight, None, out_dtype=torch.bfloat16, fp8=_fp8(self.to_kv))
        o = ewvit.attention_cross(q, kv, self.heads, self.dim_head, self.scale)
        if isinstance(self.to_out, nn.Identity):
            o = o.float()
            return o if resid is None else o + resid
        lin, drop = self.to_out[0], self.to_out[1]
        return ewvit.linear(o, lin.weight, lin.bias, drop_p=drop.p if self.training else 0.0,
                            resid=resid, out_dtype=torch.float32, fp8=_fp8(lin))


_CA_FORWARD = CrossAttention.forward


class BidirectionalCrossTransformer(nn.Module):                            # dama.py:56-78
    def __init__(self, dim, depth=1, heads=8, dim_head=64, dropout=0.):
        super().__init__()
        self.layers = nn.ModuleList([])
        for _ in range(depth):
            self.layers.append(nn.ModuleList([
                LayerNorm(dim), CrossAttention(dim, heads=heads, dim_head=dim_head, dropout=dropout),
                LayerNorm(dim), CrossAttention(dim, heads=heads, dim_head=dim_head, dropout=dropout)]))

    @staticmethod
    def _attend(att, xn, ctx, resid):
        # keep module-call semantics (hooks, a class-wide patched forward) when present
        if _hooked(att) or type(att).forward is not _CA_FORWARD:
            return resid + att(xn, ctx, kv_include_self=True)
        return att.forward_residual(xn, ctx, True, resid)

    def forward(self, space_tokens, freq_tokens):
        s, f = space_tokens.float(), freq_tokens.float()
        for s_norm, s_att, f_norm, f_att in self.layers:
            s = self._attend(s_att, s_norm(s), f, s)
            f = self._attend(f_att, f_norm(f), s, f)
        return s, f


def _spatial_mean(t):
    """mean over H, W (dama.py:165-169); over a 1x1 map the mean of one element is that
    element exactly, so no reduction launch is needed."""
    if t.shape[-2:] == (1, 1):
        return t.reshape(t.shape[0], t.shape[1])
    return t.mean(dim=[2, 3])


class FusionGate(nn.Sequential):
    """Conv3x3(2D->D, pad 1) + BN + ReLU (dama.py:124-128).  On a 1x1 map the
    zero padding leaves only the centre tap: one GEMM with W[:, :, 1, 1]; the BatchNorm
    (batch statistics over the chunk's frames) + ReLU on the ewvit BN kernel, fp32."""

    def forward(self, x):
        conv, bn, act = self[0], self[1], self[2]
        if x.shape[-2:] != (1, 1) or not x.is_cuda:
            return super().forward(x)
        B = x.shape[0]
        w = conv.weight[:, :, conv.padding[0], conv.padding[1]]
        y = ewvit.linear(x.reshape(B, -1), w, conv.bias, out_dtype=torch.float32).reshape(B, -1, 1, 1)
        if _hooked(bn) or _hooked(act) or bn.momentum is None or y.shape[1] % 8:
            return act(bn(y))
        return ewvit.batch_norm_act(y, bn, 'relu')         # BN + ReLU: one ewvit pass each way


class DAMA(nn.Module):                                                     # dama.py:80-206
    def __init__(self, in_channels=3, dim=128, num_heads=4, levels=3, batch_size=16):
        super().__init__()
        self.dim = dim
        self.levels = levels
        self.batch_size = batch_size
        self.sfe = EfficientViT(config=load_config(), channels=1280, selected_efficient_net=1,
                                feat_dim=dim, output_mode='feature_map')
        self.mwt = MWT(in_channels=in_channels, dama_dim=dim, levels=levels)
        self.gate_net = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Flatten(), Linear(2 * dim, dim // 2),
                                      nn.ReLU(), nn.Dropout(0.1), Linear(dim // 2, 3), nn.Softmax(dim=1))
        self.cross_att = BidirectionalCrossTransformer(dim=dim, depth=2, heads=num_heads,
                                                       dim_head=dim // num_heads, dropout=0.1)
        self.fusion_gate = FusionGate(nn.Conv2d(dim * 2, dim, kernel_size=3, padding=1),
                                      nn.BatchNorm2d(dim), nn.ReLU(inplace=True))

    def _gate(self, cat):
        g = self.gate_net
        if _hooked(g) or cat.shape[-2:] != (1, 1):
            return g(cat)
        l1, drop, l2 = g[2], g[4], g[5]
        h = ewvit.linear(cat.reshape(cat.shape[0], -1), l1.weight, l1.bias, act=2,
                         drop_p=drop.p if self.training else 0.0, out_dtype=torch.float32)
        return torch.softmax(ewvit.linear(h, l2.weight, l2.bias, out_dtype=torch.float32), dim=1)

    def _branches(self, frame):
        """space = sfe(frame), freq = mwt(frame) (dama.py:135-136).  The two branches are
        independent until the cross-attention, so on the GPU the MWT runs on a second
        stream: its large MFMA convs overlap the backbone's many small, latency-bound
        kernels.  Autograd replays each backward op on its forward op's stream, so the
        backward passes overlap the same way; a captured HIP graph keeps both streams."""
        if not (frame.is_cuda and _branch_streams()):
            return self.sfe(frame).float(), self.mwt(frame).float()
        main = torch.cuda.current_stream(frame.device)
        side = _side_stream(frame.device, main)
        dev = frame.device
        probe.stamp(0, dev)                # (timeline probes: no-ops unless EWVIT_PROBE=1)
        side.wait_stream(main)             # fork before the SFE work is issued on main

        if probe.ON and not getattr(self, '_probe_hooks', False):
            # slot 8: the last MWT parameter gradient accumulated (~ the MWT backward's end)
            for p in self.mwt.parameters():
                if p.requires_grad:
                    p.register_post_accumulate_grad_hook(lambda _p: probe.stamp(8, _p.device))
            # slot 10: the last SFE parameter gradient accumulated (~ the backbone backward's end)
            for p in self.sfe.parameters():
                if p.requires_grad:
                    p.register_post_accumulate_grad_hook(lambda _p: probe.stamp(10, _p.device))
            self._probe_hooks = True

        def mwt():
            with torch.cuda.stream(side), ewvit._lib.grid_cap(_mwt_grid_cap()):
                probe.stamp(2, dev)
                f = probe.tap(self.mwt(frame).float(), 5)
                probe.stamp(3, dev)
            return f
        if _MWT_FIRST:
            freq = mwt()
            space = probe.tap(self.sfe(frame).float(), 4)
            probe.stamp(1, dev)
        else:
            space = probe.tap(self.sfe(frame).float(), 4)
            probe.stamp(1, dev)
            # the MWT ops are recorded after the SFE ops: autograd runs ready backward nodes
            # latest-first, so the MWT backward is issued (on `side`) before the SFE backward
            # fills `main`, and its wait on main covers only the cross-attention backward
            freq = mwt()
        main.wait_stream(side)
        freq.record_stream(main)
        return space, freq

    def _head_fusable(self, space, freq):
        """The shape class of ewvit.head (csrc/head.hip): dim 128, 2 bidirectional layers of
        4 x 32-head cross-attention, <= 64 frames of 1x1 maps, the reference's fusion / gate
        modules, no hooks or patched forwards anywhere in the head (the tools of
        utils/visualize_feature_maps.py hook and patch them), the 12 attention Linears on one
        GEMM precision.  Returns that precision ('bf16' | 'fp8': MXFP8) or False."""
        if not (space.is_cuda and space.shape[-2:] == (1, 1) and freq.shape[-2:] == (1, 1) and self.dim == 128
                and space.shape[0] <= 64 and type(self.cross_att).forward is BidirectionalCrossTransformer.forward
                and len(self.cross_att.layers) == 2):
            return False
        precs = set()
        mods = [self.cross_att, self.fusion_gate, self.gate_net]
        for layer in self.cross_att.layers:
            mods.append(layer)
            for m in layer:
                mods.append(m)
            for att in (layer[1], layer[3]):
                if (type(att) is not CrossAttention or type(att).forward is not _CA_FORWARD or 'forward' in att.__dict__
                        or att.heads != 4 or att.dim_head != 32 or not isinstance(att.to_out, nn.Sequential)):
                    return False
                precs.update('fp8' if _fp8(t) else 'bf16' for t in (att.to_q, att.to_kv, att.to_out[0]))
                mods += [att.to_q, att.to_kv, att.to_out, att.to_out[0], att.to_out[1]]
            if not all(type(layer[j]) in (LayerNorm, nn.LayerNorm) and layer[j].normalized_shape == (128,)
                       and layer[j].elementwise_affine for j in (0, 2)):
                return False
        conv, bn = self.fusion_gate[0], self.fusion_gate[1]
        g = self.gate_net
        if (tuple(conv.weight.shape) != (128, 256, 3, 3) or conv.bias is None or conv.padding != (1, 1)
                or conv.stride != (1, 1) or conv.dilation != (1, 1) or conv.groups != 1 or bn.momentum is None
                or not bn.track_running_stats or not bn.affine or len(g) != 7 or tuple(g[2].weight.shape) != (64, 256)
                or tuple(g[5].weight.shape) != (3, 64) or g[2].bias is None or g[5].bias is None):
            return False
        mods += list(self.fusion_gate) + list(g)
        if len(precs) != 1 or any(_hooked(m) for m in mods):
            return False
        return precs.pop()

    @bf16_compute
    def _process_frame(self, frame):
        B = frame.shape[0]
        space_feats, freq_feats = self._branches(frame)
        prec = self._head_fusable(space_feats, freq_feats)
        if prec:
            # cross-attention, fusion gate, gate net and weighted sum: ewvit.head (3 launches
            # forward + backward instead of ~90; MXFP8 attention GEMMs for fp8 token GEMMs)
            drop = self.training and (self.cross_att.layers[0][1].to_out[1].p > 0 or self.gate_net[4].p > 0)
            fused, s, f = ewvit.head.dama_head(self, space_feats.reshape(B, -1), freq_feats.reshape(B, -1),
                                               ewvit.ops._seed() if drop else 0, mx=prec == 'fp8')
            return {'fused': fused, 'space': s, 'freq': f}
        Ho, Wo = space_feats.shape[-2:]
        s_flat = space_feats.flatten(2).transpose(1, 2)
        f_flat = freq_feats.flatten(2).transpose(1, 2)
        s_enh, f_enh = self.cross_att(s_flat, f_flat)
        space_feats = s_enh.transpose(1, 2).reshape(B, -1, Ho, Wo)
        freq_feats = f_enh.transpose(1, 2).reshape(B, -1, Ho, Wo)
        concat = torch.cat([space_feats, freq_feats], dim=1)
        fused_feats = self.fusion_gate(concat)
        gw = self._gate(concat)
        weighted = (gw[:, 0].view(B, 1, 1, 1) * space_feats + gw[:, 1].view(B, 1, 1, 1) * freq_feats +
                    gw[:, 2].view(B, 1, 1, 1) * fused_feats)
        return {'fused': _spatial_mean(weighted), 'space': _spatial_mean(space_feats),
                'freq': _spatial_mean(freq_feats)}

    @bf16_compute
    def forward(self, x, batch_size=16):
        B, K, C, H, W = x.shape
        if self.training and x.is_cuda:
            ewvit._lib.rng_advance(x.device)   # fresh dropout masks per step, also under graph replay
        # per-video sums over the chunks (fp32, dama.py:174-199); the reference starts from
        # zeros — 0 + s == s exactly, so the first chunk's sums are taken as they are
        acc = None
        for start in range(0, K, batch_size):
            end = min(start + batch_size, K)
            feats = self._process_frame(x[:, start:end].flatten(0, 1))
            part = {k: feats[k].float().view(B, -1, self.dim).sum(dim=1) for k in ('fused', 'space', 'freq')}
            acc = part if acc is None else {k: acc[k] + part[k] for k in acc}
        return {k: acc[k] / K for k in ('fused', 'space', 'freq')}
