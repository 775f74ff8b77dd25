"""ORACLE (test infrastructure only) — torch fp32 CPU eager restatement of the
reference hot path, module tree and state-dict keys identical to the reference.

Each class cites the reference lines it restates.  Third-party numerics:
``DWT`` restates pytorch_wavelets DWTForward(J=1,'haar','zero') (see oracle/dwt.py
for the arithmetic, pinned by pywt), the backbone is oracle.effnetv2.
"""
import math

import numpy as np
import torch
from torch import nn
from torch.nn import functional as F

from .effnetv2 import efficientnet_v2_s

# config/architecture.yaml of the reference (values, not a file read)
ARCH_CONFIG = {'model': {'image-size': 224, 'patch-size': 7, 'num-classes': 1, 'dim': 512,
                         'depth': 2, 'dim-head': 64, 'heads': 8, 'mlp-dim': 2048,
                         'emb-dim': 64, 'dropout': 0.15, 'emb-dropout': 0.15}}

_S = float(np.float32(0.7071067811865476))


class DWTForward(nn.Module):
    """pytorch_wavelets.DWTForward(J=1, wave='haar', mode='zero') — AFB2D as two
    grouped stride-2 conv2d (row pass dim 3, then column pass dim 2).  Buffers
    named as pytorch_wavelets registers them (h0_col, h1_col, h0_row, h1_row)."""

    def __init__(self):
        super().__init__()
        h0 = torch.tensor([_S, _S], dtype=torch.float32)
        h1 = torch.tensor([_S, -_S], dtype=torch.float32)
        self.register_buffer('h0_col', h0.reshape(1, 1, 2, 1))
        self.register_buffer('h1_col', h1.reshape(1, 1, 2, 1))
        self.register_buffer('h0_row', h0.reshape(1, 1, 1, 2))
        self.register_buffer('h1_row', h1.reshape(1, 1, 1, 2))

    @staticmethod
    def _afb1d(x, h0, h1, dim):
        C = x.shape[1]
        N = x.shape[dim]
        if N % 2 == 1:
            x = F.pad(x, (0, 0, 0, 1) if dim == 2 else (0, 1, 0, 0))
        h = torch.cat([h0, h1] * C, dim=0)
        stride = (2, 1) if dim == 2 else (1, 2)
        return F.conv2d(x, h, stride=stride, groups=C)

    def forward(self, x):
        lohi = self._afb1d(x, self.h0_row, self.h1_row, 3)
        y = self._afb1d(lohi, self.h0_col, self.h1_col, 2)
        s = y.shape
        y = y.reshape(s[0], -1, 4, s[-2], s[-1])
        return y[:, :, 0].contiguous(), [y[:, :, 1:].contiguous()]


def _cbr(cin, cout, stride=1):
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, stride=stride),
                         nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class MWT(nn.Module):
    """network/mwt.py:7-119."""

    def __init__(self, in_channels=3, dama_dim=128, levels=3):
        super().__init__()
        self.in_channels, self.dama_dim, self.levels = in_channels, dama_dim, levels
        self.dwt = DWTForward()                                              # mwt.py:20
        self.freq_conv = _cbr(dama_dim, dama_dim, stride=2)                  # mwt.py:23-36
        self.freq_pool = nn.Sequential(nn.MaxPool2d(2, 2),                   # mwt.py:38-44
                                       nn.Conv2d(dama_dim, dama_dim, 3, padding=1, stride=2),
                                       nn.BatchNorm2d(dama_dim), nn.ReLU(inplace=True),
                                       nn.AdaptiveAvgPool2d(1))
        self.hf_conv = nn.ModuleDict({                                       # mwt.py:47-65
            'seperate': nn.ModuleList([_cbr(in_channels, 6 * in_channels) for _ in range(3)]),
            'fusion': _cbr(18 * in_channels, dama_dim)})
        self.multiscale_fusion = _cbr(levels * dama_dim, dama_dim)           # mwt.py:68-72

    def wavelet_transform(self, x, target_size):                             # mwt.py:74-90
        B, C, H, W = x.shape
        ll, hf = self.dwt(x)
        hf = hf[0].reshape(B, 3 * C, H // 2, W // 2)
        if self.levels > 1:
            hf = F.interpolate(hf, size=target_size, mode='bilinear')
        processed = [self.hf_conv['seperate'][i](hf[:, i * C:(i + 1) * C]) for i in range(3)]
        return ll, self.hf_conv['fusion'](torch.cat(processed, dim=1))

    def forward(self, x):                                                    # mwt.py:92-119
        B, C, H, W = x.shape
        target = (H // 2, W // 2)
        cur, highs = x, []
        for _ in range(self.levels):
            ll, hf = self.wavelet_transform(cur, target)
            highs.append(hf)
            cur = ll
        f = self.multiscale_fusion(torch.cat(highs, dim=1))
        return self.freq_pool(self.freq_conv(f))


class PreNorm(nn.Module):                                                    # sfe.py:20-27
    def __init__(self, dim, fn):
        super().__init__()
        self.norm = nn.LayerNorm(dim)
        self.fn = fn

    def forward(self, x, **kw):
        return self.fn(self.norm(x), **kw)


class FeedForward(nn.Module):                                                # sfe.py:29-40
    def __init__(self, dim, hidden_dim, dropout=0.):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(dim, hidden_dim), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hidden_dim, dim), nn.Dropout(dropout))

    def forward(self, x):
        return self.net(x)


def _split_heads(t, h):
    b, n, hd = t.shape
    return t.reshape(b, n, h, hd // h).transpose(1, 2)


def _merge_heads(t):
    b, h, n, d = t.shape
    return t.transpose(1, 2).reshape(b, n, h * d)


class Attention(nn.Module):                                                  # sfe.py:42-70
    def __init__(self, dim, heads=8, dim_head=64, dropout=0.):
        super().__init__()
        inner = dim_head * heads
        project_out = not (heads == 1 and dim_head == dim)
        self.heads = heads
        self.scale = dim_head ** -0.5
        self.attend = nn.Softmax(dim=-1)
        self.to_qkv = nn.Linear(dim, inner * 3, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(dropout)) if project_out else nn.Identity()

    def forward(self, x):
        q, k, v = (_split_heads(t, self.heads) for t in self.to_qkv(x).chunk(3, dim=-1))
        dots = torch.einsum('bhid,bhjd->bhij', q, k) * self.scale
        out = torch.einsum('bhij,bhjd->bhid', self.attend(dots), v)
        return self.to_out(_merge_heads(out))


class Transformer(nn.Module):                                                # sfe.py:72-85
    def __init__(self, dim, depth, heads, dim_head, mlp_dim, dropout=0.):
        super().__init__()
        self.layers = nn.ModuleList([nn.ModuleList([
            PreNorm(dim, Attention(dim, heads=heads, dim_head=dim_head, dropout=dropout)),
            PreNorm(dim, FeedForward(dim, mlp_dim, dropout=0))]) for _ in range(depth)])

    def forward(self, x):
        for attn, ff in self.layers:
            x = attn(x) + x
            x = ff(x) + x
        return x


class EfficientViT(nn.Module):                                               # sfe.py:87-173
    """selected_efficient_net=1 (torchvision v2_s) path only — the one DAMA builds."""

    def __init__(self, config=ARCH_CONFIG, channels=1280, selected_efficient_net=1, feat_dim=128,
                 output_mode='feature_map'):
        super().__init__()
        m = config['model']
        self.output_mode = output_mode
        self.selected_efficient_net = selected_efficient_net
        self.efficient_net = efficientnet_v2_s()
        self.efficient_net.classifier = nn.Identity()
        for i, (_, p) in enumerate(self.efficient_net.named_parameters()):   # sfe.py:115-119
            p.requires_grad = i > 5
        p = m['patch-size']
        dim = m['dim']
        self.patch_size = p
        self.pos_embedding = nn.Parameter(torch.randn(m['emb-dim'], 1, dim))
        self.patch_to_embedding = nn.Linear(channels * p * p, dim)
        self.cls_token = nn.Parameter(torch.randn(1, 1, dim))
        self.dropout = nn.Dropout(m['emb-dropout'])
        self.transformer = Transformer(dim, m['depth'], m['heads'], m['dim-head'], m['mlp-dim'], m['dropout'])
        self.to_cls_token = nn.Identity()
        self.mlp_head = nn.Sequential(nn.Linear(dim, m['mlp-dim']), nn.ReLU(), nn.Linear(m['mlp-dim'], m['num-classes']))
        self.feat_map = nn.Sequential(nn.Linear(dim, feat_dim), nn.ReLU())

    def head(self, x):
        """sfe.py:153-173 from the backbone map x [B,1280,h,w]."""
        p = self.patch_size
        b, c, hh, ww = x.shape
        # rearrange 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)'
        y = x.reshape(b, c, hh // p, p, ww // p, p).permute(0, 2, 4, 3, 5, 1).reshape(b, (hh // p) * (ww // p), p * p * c)
        y = self.patch_to_embedding(y)
        x = torch.cat((self.cls_token.expand(b, -1, -1), y), 1)
        x = x + self.pos_embedding[0:b]
        x = self.dropout(x)
        x = self.transformer(x)
        if self.output_mode == 'cls':
            return self.mlp_head(self.to_cls_token(x[:, 0]))
        B, N, D = x.shape
        H = W = int(math.sqrt(N - 1))
        x = self.feat_map(x[:, 1:])
        return x.reshape(B, H, W, -1).permute(0, 3, 1, 2)

    def forward(self, img):
        return self.head(self.efficient_net.features(img))


class CrossAttention(nn.Module):                                             # dama.py:15-53
    def __init__(self, dim, heads=8, dim_head=64, dropout=0.):
        super().__init__()
        inner = dim_head * heads
        project_out = not (heads == 1 and dim_head == dim)
        self.heads = heads
        self.scale = dim_head ** -0.5
        self.attend = nn.Softmax(dim=-1)
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(dim, inner * 2, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(dropout)) if project_out else nn.Identity()

    def forward(self, x, context=None, kv_include_self=False):
        context = context if context is not None else x
        if kv_include_self:
            context = torch.cat((x, context), dim=1)
        q = _split_heads(self.to_q(x), self.heads)
        k, v = (_split_heads(t, self.heads) for t in self.to_kv(context).chunk(2, dim=-1))
        dots = torch.einsum('bhid,bhjd->bhij', q, k) * self.scale
        out = torch.einsum('bhij,bhjd->bhid', self.attend(dots), v)
        return self.to_out(_merge_heads(out))


class BidirectionalCrossTransformer(nn.Module):                              # dama.py:56-78
    def __init__(self, dim, depth=1, heads=8, dim_head=64, dropout=0.):
        super().__init__()
        self.layers = nn.ModuleList([nn.ModuleList([
            nn.LayerNorm(dim), CrossAttention(dim, heads, dim_head, dropout),
            nn.LayerNorm(dim), CrossAttention(dim, heads, dim_head, dropout)]) for _ in range(depth)])

    def forward(self, s, f):
        for sn, s_att, fn, f_att in self.layers:
            s = s + s_att(sn(s), f, kv_include_self=True)
            f = f + f_att(fn(f), s, kv_include_self=True)
        return s, f


class DAMA(nn.Module):                                                       # dama.py:80-206
    def __init__(self, in_channels=3, dim=128, num_heads=4, levels=3, batch_size=16, config=ARCH_CONFIG):
        super().__init__()
        self.dim, self.levels, self.batch_size = dim, levels, batch_size
        self.sfe = EfficientViT(config, channels=1280, selected_efficient_net=1, feat_dim=dim,
                                output_mode='feature_map')
        self.mwt = MWT(in_channels=in_channels, dama_dim=dim, levels=levels)
        self.gate_net = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(2 * dim, dim // 2),
                                      nn.ReLU(), nn.Dropout(0.1), nn.Linear(dim // 2, 3), nn.Softmax(dim=1))
        self.cross_att = BidirectionalCrossTransformer(dim, depth=2, heads=num_heads,
                                                       dim_head=dim // num_heads, dropout=0.1)
        self.fusion_gate = nn.Sequential(nn.Conv2d(dim * 2, dim, 3, padding=1), nn.BatchNorm2d(dim),
                                         nn.ReLU(inplace=True))

    def fuse(self, space_feats, freq_feats):
        """dama.py:139-169 given the two branch outputs [B,D,h,w]."""
        B = space_feats.shape[0]
        Ho, Wo = space_feats.shape[-2:]
        sf = space_feats.flatten(2).transpose(1, 2)
        ff = freq_feats.flatten(2).transpose(1, 2)
        se, fe = self.cross_att(sf, ff)
        space_feats = se.transpose(1, 2).reshape(B, -1, Ho, Wo)
        freq_feats = fe.transpose(1, 2).reshape(B, -1, Ho, Wo)
        cat = torch.cat([space_feats, freq_feats], dim=1)
        fused = self.fusion_gate(cat)
        g = self.gate_net(cat)
        w = g[:, 0].view(B, 1, 1, 1) * space_feats + g[:, 1].view(B, 1, 1, 1) * freq_feats + \
            g[:, 2].view(B, 1, 1, 1) * fused
        return {'fused': w.mean(dim=[2, 3]), 'space': space_feats.mean(dim=[2, 3]),
                'freq': freq_feats.mean(dim=[2, 3])}

    def _process_frame(self, frame):
        return self.fuse(self.sfe(frame), self.mwt(frame))

    def forward(self, x, batch_size=16):                                     # dama.py:171-206
        B, K, C, H, W = x.shape
        acc = {k: torch.zeros(B, self.dim, device=x.device) for k in ('fused', 'space', 'freq')}
        for s in range(0, K, batch_size):
            e = min(s + batch_size, K)
            feats = self._process_frame(x[:, s:e].flatten(0, 1))
            for k in acc:
                acc[k] = acc[k] + feats[k].view(B, -1, self.dim).sum(dim=1)
        return {k: v / K for k, v in acc.items()}


class DeepfakeDetector(nn.Module):                                           # model.py:9-99 (dynamic)
    def __init__(self, in_channels=3, dama_dim=128, batch_size=16, ablation='dynamic'):
        super().__init__()
        self.dama_dim, self.in_channels, self.batch_size = dama_dim, in_channels, batch_size
        self.ablation = ablation
        self.dama = DAMA(in_channels, dama_dim, num_heads=4, levels=3, batch_size=batch_size)
        self.classifier = nn.Sequential(nn.Linear(dama_dim, 64), nn.ReLU(), nn.Dropout(0.3), nn.Linear(64, 1))

    def forward(self, x, batch_size, ablation):
        if batch_size is not None:
            self.batch_size = batch_size
        d = self.dama(x, batch_size=self.batch_size)
        return {'logits': self.classifier(d['fused']), 'fused': d['fused'], 'space': d['space'],
                'freq': d['freq']}


def orthogonal_loss(space_feats, freq_feats):                                # train.py:55-67
    _, D = space_feats.shape
    s = F.normalize(space_feats, p=2, dim=1)
    f = F.normalize(freq_feats, p=2, dim=1)
    cov = s.T @ f
    off = cov * (1 - torch.eye(D, device=cov.device))
    return torch.norm(off, p='fro') ** 2 / (D * (D - 1))


def combined_loss(outputs, labels, criterion, epoch, max_epochs):            # train.py:69-91
    logits = outputs['logits']
    labels = labels.view(-1, 1).float()
    cls = criterion(logits, labels)
    if epoch < 0.2 * max_epochs:
        return cls
    lam = min(1.0, (epoch - 0.2 * max_epochs) / (0.5 * max_epochs))
    return cls + lam * orthogonal_loss(outputs['space'], outputs['freq'])
