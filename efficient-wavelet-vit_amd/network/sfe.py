"""Spatial feature extractor — drop-in for reference network/sfe.py:12-173.

EfficientNetV2-S backbone -> one 7x7 patch -> patch_to_embedding -> CLS + pos
embedding -> pre-norm ViT (depth 2) -> feat_map.  On MI355X every linear layer,
LayerNorm and the n=2-token attention run on the ewvit kernels:
* to_qkv (bf16 out) -> short-sequence attention -> to_out with dropout and the
  residual add fused into the GEMM epilogue;
* FeedForward: Linear+GELU fused (pre-activation kept for backward) -> Linear
  with the residual fused;
* patch_to_embedding: split-K GEMM over K = 62720 straight from the channels-last
  backbone map (the 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)' rearrange of
  sfe.py:153 is a view of NHWC memory when the map is one patch).
Module/attribute/state-dict names are the reference's.
"""
import math

import torch
from torch import nn
from torch.nn import functional as F

import ewvit
from ewvit import probe

from . import bf16_compute
from .efficientnet import efficientnet_v2_s


def _cdt():
    return torch.get_autocast_dtype('cuda') if torch.is_autocast_enabled('cuda') else torch.float32


def _hooked(m):
    return bool(m._forward_hooks or m._forward_pre_hooks or m._backward_hooks)


def _fp8(m):
    """True when network.set_gemm_precision put this Linear's GEMMs on fp8 e4m3."""
    return getattr(m, 'gemm_precision', 'bf16') == 'fp8'


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm on the ewvit kernel; output in `out_dtype` (default: fp32)."""

    out_dtype = torch.float32

    def forward(self, x):
        return ewvit.layer_norm(x, self.weight, self.bias, self.eps, out_dtype=self.out_dtype)


class Linear(nn.Linear):
    """nn.Linear on the ewvit MFMA GEMM (fp32 master weights read directly)."""

    def forward(self, x):
        return ewvit.linear(x, self.weight, self.bias, out_dtype=torch.float32, fp8=_fp8(self))


class Residual(nn.Module):                                                 # sfe.py:12-18
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x, **kwargs):
        return self.fn(x, **kwargs) + x


class PreNorm(nn.Module):                                                  # sfe.py:20-27
    def __init__(self, dim, fn):
        super().__init__()
        self.norm = LayerNorm(dim)
        self.fn = fn

    def forward(self, x, **kwargs):
        return self.fn(self.norm(x), **kwargs)

    def forward_residual(self, x):
        """fn(norm(x)) + x with the add fused into fn's last GEMM."""
        if _hooked(self) or _hooked(self.fn) or not hasattr(self.fn, 'forward_residual'):
            return self(x) + x
        return self.fn.forward_residual(self.norm(x), x)


class FeedForward(nn.Module):                                              # sfe.py:29-40
    def __init__(self, dim, hidden_dim, dropout=0.):
        super().__init__()
        self.net = nn.Sequential(Linear(dim, hidden_dim), nn.GELU(), nn.Dropout(dropout),
                                 Linear(hidden_dim, dim), nn.Dropout(dropout))

    def _p(self, i):
        return self.net[i].p if self.training else 0.0

    def forward(self, x):
        return self.forward_residual(x, None)

    def forward_residual(self, x, resid):
        l1, l2 = self.net[0], self.net[3]
        h = ewvit.linear(x, l1.weight, l1.bias, act=1, drop_p=self._p(2), out_dtype=torch.bfloat16, fp8=_fp8(l1))
        return ewvit.linear(h, l2.weight, l2.bias, drop_p=self._p(4), resid=resid, out_dtype=torch.float32,
                            fp8=_fp8(l2))


class Attention(nn.Module):                                                # sfe.py:42-70
    def __init__(self, dim, heads=8, dim_head=64, dropout=0.):
        super().__init__()
        inner_dim = dim_head * heads
        project_out = not (heads == 1 and dim_head == dim)
        self.heads = heads
        self.dim_head = dim_head
        self.scale = dim_head ** -0.5
        self.attend = nn.Softmax(dim=-1)
        self.to_qkv = Linear(dim, inner_dim * 3, bias=False)
        self.to_out = nn.Sequential(Linear(inner_dim, dim), nn.Dropout(dropout)) if project_out else nn.Identity()

    def forward(self, x):
        return self.forward_residual(x, None)

    def forward_residual(self, x, resid):
        qkv = ewvit.linear(x, self.to_qkv.weight, None, out_dtype=torch.bfloat16, fp8=_fp8(self.to_qkv))
        o = ewvit.attention_packed(qkv, self.heads, self.dim_head, self.scale)
        if isinstance(self.to_out, nn.Identity):
            o = o.float()
            return o if resid is None else o + resid
        lin, drop = self.to_out[0], self.to_out[1]
        return ewvit.linear(o, lin.weight, lin.bias, drop_p=drop.p if self.training else 0.0,
                            resid=resid, out_dtype=torch.float32, fp8=_fp8(lin))


class Transformer(nn.Module):                                              # sfe.py:72-85
    def __init__(self, dim, depth, heads, dim_head, mlp_dim, dropout=0.):
        super().__init__()
        self.layers = nn.ModuleList([])
        for _ in range(depth):
            self.layers.append(nn.ModuleList([
                PreNorm(dim, Attention(dim, heads=heads, dim_head=dim_head, dropout=dropout)),
                PreNorm(dim, FeedForward(dim=dim, hidden_dim=mlp_dim, dropout=0))]))

    def forward(self, x):
        x = x.float()
        fused = [_vit_fusable(attn, ff, x) for attn, ff in self.layers]     # None | 'bf16' | 'fp8'
        slot = {}
        for prec in ('bf16', 'fp8'):
            sel = [i for i, f in enumerate(fused) if f == prec][:ewvit.vit.PACK_MAX]
            if sel:
                # the fused layers' GEMM weights (both orientations; bf16, or MXFP8 for fp8 token
                # GEMMs), one launch per precision (ewvit.vit.pack)
                mx = prec == 'fp8'
                packed = ewvit.vit.pack([tuple(self.layers[i]) for i in sel], mx=mx)
                slot.update({i: (packed, k, mx) for k, i in enumerate(sel)})
        for i, (attn, ff) in enumerate(self.layers):
            if i in slot:
                # the layer on csrc/vit.hip: 4 launches forward, 5 backward (ewvit.vit)
                x = ewvit.vit.vit_layer(attn, ff, x, self.training, *slot[i])
                continue
            x = attn.forward_residual(x)
            x = ff.forward_residual(x)
        return x



def _vit_fusable(attn, ff, x):
    """The shape class of ewvit.vit (csrc/vit.hip): dim 512, 8 heads of 64, mlp 2048, 2 tokens
    per frame, <= 64 frames, the reference's module structure (no hooks or patched forwards,
    the FeedForward's dropouts 0 or eval), the four Linears on one GEMM precision.  Returns
    that precision ('bf16' | 'fp8': MXFP8, network.set_gemm_precision) or None."""
    if torch.compiler.is_compiling():        # traced (torch.compile): the custom-op module path
        return None
    if not (ewvit.vit.enabled() and x.is_cuda and x.dim() == 3 and x.shape[1] == 2 and x.shape[2] == 512
            and 1 <= x.shape[0] <= 64):
        return False
    if type(attn) is not PreNorm or type(ff) is not PreNorm:
        return False
    a, f = attn.fn, ff.fn
    if (type(a) is not Attention or type(f) is not FeedForward or 'forward' in a.__dict__ or 'forward' in f.__dict__
            or type(a).forward_residual is not Attention.forward_residual or a.heads != 8 or a.dim_head != 64
            or not isinstance(a.to_out, nn.Sequential) or len(f.net) != 5
            or not isinstance(f.net[1], nn.GELU) or f.net[1].approximate != 'none'):
        return False
    lins = (a.to_qkv, a.to_out[0], f.net[0], f.net[3])
    if any(type(m) is not Linear for m in lins) or a.to_qkv.bias is not None:
        return False
    prec = {('fp8' if _fp8(m) else 'bf16') for m in lins}
    if len(prec) != 1:
        return False
    if (tuple(a.to_qkv.weight.shape) != (1536, 512) or tuple(a.to_out[0].weight.shape) != (512, 512)
            or tuple(f.net[0].weight.shape) != (2048, 512) or tuple(f.net[3].weight.shape) != (512, 2048)):
        return False
    norms = (attn.norm, ff.norm)
    if any(type(n) not in (LayerNorm, nn.LayerNorm) or n.normalized_shape != (512,) or not n.elementwise_affine
           for n in norms) or attn.norm.eps != ff.norm.eps:
        return False
    if ff.training and (f.net[2].p > 0 or f.net[4].p > 0):
        return False
    ts = [attn.norm.weight, attn.norm.bias, a.to_qkv.weight, a.to_out[0].weight, a.to_out[0].bias, ff.norm.weight,
          ff.norm.bias, f.net[0].weight, f.net[0].bias, f.net[3].weight, f.net[3].bias]
    if any(t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda for t in ts):
        return False
    mods = [attn, ff, a, f, attn.norm, ff.norm, a.to_qkv, a.to_out, *a.to_out, *f.net]
    return None if any(_hooked(m) for m in mods) else prec.pop()


class EfficientViT(nn.Module):                                             # sfe.py:87-173
    def __init__(self, config, channels=512, selected_efficient_net=0, feat_dim=128, output_mode=None):
        super().__init__()
        self.output_mode = output_mode
        m = config['model']
        image_size, patch_size = m['image-size'], m['patch-size']
        dim, depth, heads = m['dim'], m['depth'], m['heads']
        mlp_dim, emb_dim, dim_head = m['mlp-dim'], m['emb-dim'], m['dim-head']
        dropout, emb_dropout = m['dropout'], m['emb-dropout']
        num_classes = m['num-classes']
        assert image_size % patch_size == 0, 'image dimensions must be divisible by the patch size'
        self.selected_efficient_net = selected_efficient_net
        if selected_efficient_net == 0:
            raise NotImplementedError(
                'EfficientNet-b0 (efficientnet_pytorch.from_pretrained, sfe.py:109) is only used by the '
                "out-of-scope 'sfe_only'/'sfe_mwt' ablations and needs a network fetch")
        self.efficient_net = efficientnet_v2_s(weights=None)
        self.efficient_net.classifier = nn.Identity()
        for index, (_, param) in enumerate(self.efficient_net.named_parameters()):  # sfe.py:115-119
            param.requires_grad = index > 5
        self.patch_size = patch_size
        self.pos_embedding = nn.Parameter(torch.randn(emb_dim, 1, dim))
        self.patch_to_embedding = Linear(channels * patch_size ** 2, dim)
        self.cls_token = nn.Parameter(torch.randn(1, 1, dim))
        self.dropout = nn.Dropout(emb_dropout)
        self.transformer = Transformer(dim, depth, heads, dim_head, mlp_dim, dropout)
        self.to_cls_token = nn.Identity()
        self.mlp_head = nn.Sequential(Linear(dim, mlp_dim), nn.ReLU(), Linear(mlp_dim, num_classes))
        self.feat_map = nn.Sequential(Linear(dim, feat_dim), nn.ReLU())

    def patches(self, x):
        """'b c (h p1) (w p2) -> b (h w) (p1 p2 c)' (sfe.py:153) — a view for a
        channels-last single-patch map."""
        p = self.patch_size
        b, c, hh, ww = x.shape
        t = x.permute(0, 2, 3, 1)
        if hh == p and ww == p:
            return t.reshape(b, 1, p * p * c)
        return t.reshape(b, hh // p, p, ww // p, p, c).permute(0, 1, 3, 2, 4, 5).reshape(b, (hh // p) * (ww // p), p * p * c)

    def head(self, x):
        """sfe.py:153-173 from the backbone map x [B, C, h, w]."""
        B = x.shape[0]
        P = self.pos_embedding.shape[0]
        if B > P and P != 1:
            # pos_embedding[0:B] has P rows, which broadcast against B frames only when P == 1
            raise RuntimeError(f'EfficientViT: {B} frames in one chunk exceed pos_embedding rows '
                               f'({P}) — the reference fails here too (sfe.py:158-159)')
        y = self.patches(x)
        pe = self.patch_to_embedding
        y = ewvit.linear(y, pe.weight, pe.bias, out_dtype=torch.float32, fp8=_fp8(pe))
        if (ewvit.vit.enabled() and y.shape[1:] == (1, 512) and self.cls_token.shape == (1, 1, 512)
                and self.pos_embedding.shape[1:] == (1, 512) and B <= P <= 64
                and type(self.dropout) is nn.Dropout
                and not _hooked(self.dropout) and not torch.compiler.is_compiling()):
            # CLS concat + pos_embedding[0:B] + emb dropout in one launch (ewvit.vit.embed)
            tok = ewvit.vit.embed(y, self.cls_token, self.pos_embedding, self.dropout.p if self.training else 0.0)
        else:
            tok = torch.cat((self.cls_token.expand(B, -1, -1), y), 1) + self.pos_embedding[0:B]
            tok = self.dropout(tok)
        tok = self.transformer(tok)
        if self.output_mode == 'cls':
            return self.mlp_head(self.to_cls_token(tok[:, 0]))
        Bn, N, D = tok.shape
        H = W = int(math.sqrt(N - 1))
        fm = self.feat_map[0]
        f = ewvit.linear(tok[:, 1:], fm.weight, fm.bias, act=2, out_dtype=torch.float32, fp8=_fp8(fm))
        return f.reshape(Bn, H, W, -1).permute(0, 3, 1, 2)

    @bf16_compute
    def forward(self, img, mask=None):
        f = self.efficient_net.features(img)
        probe.stamp(7, f.device)           # (timeline probes: no-ops unless EWVIT_PROBE=1)
        return self.head(probe.tap(f, 6))
