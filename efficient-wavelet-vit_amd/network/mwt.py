"""MWT — multi-level wavelet branch (drop-in for reference network/mwt.py:7-119).

Hot path on MI355X:
* one ewvit kernel pair replaces the per-level DWT + reshape + bilinear upsample
  (mwt.py:76-81): ``dwt_haar_fwd`` reads the frames once and emits every level's
  bands, ``hf_upsample`` writes all levels' upsampled HF input channels-last
  ``[L, N, H/2, W/2, 3C]`` (channel c*3+band, mwt.py:77);
* the three ``hf_conv['seperate'][i]`` convs (colour channel i's three bands,
  mwt.py:84-86) run as ONE grouped conv (groups=3) over all levels at once
  (weights are shared by the levels, mwt.py:108), likewise ``hf_conv['fusion']``;
  BatchNorm statistics and running-stat updates stay per level and in the
  reference's order, so train-mode numerics and state are the reference's;
* the fusion / multiscale / freq convs run on the ewvit MFMA implicit-GEMM conv
  (csrc/conv.hip); multiscale_fusion reads the level-major fusion outputs as their
  channel concatenation in place (no torch.cat of mwt.py:112 in HBM);
* BatchNorm + ReLU are one fused ewvit pass (csrc/batchnorm.hip).
The seperate conv (9 band channels, zero-padded to 16 by the upsample pass -> 54
channels, zero-padded to 64) runs as the grouped conv it is on csrc/hfsep.hip, its
BatchNorm statistics summed in the same pass (ewvit.hfsep); fp32 / other shapes take one
block-diagonal conv.

If ``wavelet_transform`` is overridden on the instance or class (as
utils/visualize_feature_maps.py:151-158 does), forward falls back to the
reference's per-level loop calling ``self.wavelet_transform`` (still on GPU).
"""
import os

import torch
from torch import nn
from torch.nn import functional as F

import ewvit

from . import bf16_compute


class DWTForward(nn.Module):
    """pytorch_wavelets.DWTForward(J, wave='haar', mode='zero') on the ewvit DWT kernel.
    Same buffers (h0_col, h1_col, h0_row, h1_row) for state-dict compatibility."""

    def __init__(self, J=1, wave='haar', mode='zero'):
        super().__init__()
        if wave != 'haar' or mode != 'zero':
            raise NotImplementedError('ewvit DWT implements haar / zero padding only (mwt.py:20)')
        self.J = J
        s = 0.7071067811865476
        h0 = torch.tensor([s, s], dtype=torch.float32)
        h1 = torch.tensor([s, -s], dtype=torch.float32)
        self.register_buffer('h0_col', h0.reshape(1, 1, 2, 1))
        self.register_buffer('h1_col', h1.reshape(1, 1, 2, 1))
        self.register_buffer('h0_row', h0.reshape(1, 1, 1, 2))
        self.register_buffer('h1_row', h1.reshape(1, 1, 1, 2))

    def forward(self, x):
        odt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        return ewvit.dwt_haar(x, self.J, out_dtype=odt)


class Conv3x3(nn.Conv2d):
    """nn.Conv2d(k=3, pad=1) on the ewvit MFMA implicit-GEMM kernels (csrc/conv.hip)
    for channels-last inputs whose channel count is a multiple of 8 (extra input
    channels beyond in_channels must be zero padding); other inputs (the 3-channel
    per-level path of `wavelet_transform`) go to the library conv.
    ``levels > 1``: x is level-major [levels*B, C, H, W] and the conv input is
    cat(x.chunk(levels), dim=1), read in place by the kernel."""

    def forward(self, x, levels=1):
        C = x.shape[1] * levels
        if x.is_cuda and C % 8 == 0 and C >= self.in_channels and self.out_channels % 8 == 0 and \
                (levels == 1 or (x.shape[1] % 32 == 0 and C == self.in_channels)):
            return ewvit.conv2d(x, self.weight, self.bias, self.stride[0], levels)
        if levels > 1:
            x = torch.cat(x.chunk(levels), dim=1)
        return super().forward(x[:, :self.in_channels])


def _fusable(bn, y):
    return y.is_cuda and y.shape[1] % 8 == 0 and y.shape[1] <= 2048 and not (bn._forward_hooks or bn._forward_pre_hooks)


def _epi_stats(conv, bn, x, levels=1, groups=1):
    """Conv with the BatchNorm batch statistics summed in its epilogue ->
    (y, partials) for ewvit.batch_norm_act, or None (the plain conv + BN path)."""
    if (type(conv) is not Conv3x3 or not bn.training or not bn.track_running_stats or bn.momentum is None
            or conv._forward_hooks or conv._forward_pre_hooks or bn._forward_hooks or bn._forward_pre_hooks
            or not x.is_cuda or bn.num_features > 2048):
        return None
    r = ewvit.conv.conv2d_bn_stats(x, conv.weight, conv.bias, conv.stride[0], bn.running_mean, levels, groups)
    return None if r is None else (r[0], r[1:])


# the hf_conv['fusion'] BatchNorm + ReLU applied inside multiscale_fusion's conv (ewvit.conv.
# BnReluConvFn) instead of by its own pass (0: the separate apply pass, A/B and tests)
_FOLD_FUSION_BN = os.environ.get('EWVIT_FOLD_FUSION_BN', '1') != '0'


class PendingBNReLU:
    """A training BatchNorm(+ReLU) output not yet materialised: the producer's raw output z,
    the batch statistics its epilogue summed, the CBR whose BN / ReLU it is and the BN groups
    (levels).  The consumer either folds it into its conv (CBR.forward -> ewvit.conv.
    bn_relu_conv2d_bn_stats) or calls materialize()."""
    __slots__ = ('z', 'partials', 'cbr', 'groups')

    def __init__(self, z, partials, cbr, groups):
        self.z, self.partials, self.cbr, self.groups = z, partials, cbr, groups

    def materialize(self):
        return ewvit.batch_norm_act(self.z, self.cbr[1], 'relu', groups=self.groups, partials=self.partials)


class CBR(nn.Sequential):
    """Conv3x3 -> BatchNorm2d -> ReLU; BN + ReLU as one fused ewvit pass, its batch
    statistics summed in the conv's epilogue where the conv kernel allows.
    ``levels``: see Conv3x3.forward.  x may be a PendingBNReLU (the level-major hf fusion
    output, levels groups): its BatchNorm + ReLU then run inside this conv's operand reads."""

    def _fold(self, p, levels):
        conv, bn = self[0], self[1]
        src_bn = p.cbr[1]
        if not (p.groups == levels and type(conv) is Conv3x3 and bn.training and bn.track_running_stats
                and bn.momentum is not None and conv.stride[0] == 1 and conv.padding[0] == 1
                and not (conv._forward_hooks or conv._forward_pre_hooks or bn._forward_hooks or bn._forward_pre_hooks)
                and conv.weight.requires_grad and src_bn.weight is not None and src_bn.weight.requires_grad
                and ewvit.conv.bn_relu_ok(p.z, conv.weight, levels)):
            return None
        r = ewvit.conv.bn_relu_conv2d_bn_stats(p.z, p.partials, src_bn, conv.weight, conv.bias, bn.running_mean,
                                               levels)
        return r[0], r[1:]

    def forward(self, x, levels=1):
        if isinstance(x, PendingBNReLU):
            r = self._fold(x, levels)
            if r is not None:
                return ewvit.batch_norm_act(r[0], self[1], 'relu', partials=r[1])
            x = x.materialize()
        r = _epi_stats(self[0], self[1], x, levels)
        if r is not None:
            return ewvit.batch_norm_act(r[0], self[1], 'relu', partials=r[1])
        y = self[0](x, levels) if levels > 1 else self[0](x)
        if _fusable(self[1], y):
            return ewvit.batch_norm_act(y, self[1], 'relu')
        return self[2](self[1](y))


class FreqPool(nn.Sequential):
    """MaxPool2d(2) -> Conv3x3 s2 -> BatchNorm2d -> ReLU -> AdaptiveAvgPool2d(1) (mwt.py:38-44)."""

    def forward(self, x):
        mp = self[0]
        if (x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32)
                and mp.kernel_size in (2, (2, 2)) and mp.stride in (2, (2, 2)) and mp.padding in (0, (0, 0))
                and mp.dilation in (1, (1, 1)) and not mp.ceil_mode and not mp.return_indices
                and not (mp._forward_hooks or mp._forward_pre_hooks)):
            p = ewvit.maxpool2(x)               # csrc/pool.hip
        else:
            p = mp(x)
        r = _epi_stats(self[1], self[2], p)
        if r is not None:
            return self[4](ewvit.batch_norm_act(r[0], self[2], 'relu', partials=r[1]))
        y = self[1](p)
        y = ewvit.batch_norm_act(y, self[2], 'relu') if _fusable(self[2], y) else self[3](self[2](y))
        return self[4](y)


def _cbr(cin, cout, stride=1, conv=Conv3x3):
    return CBR(conv(cin, cout, 3, padding=1, stride=stride), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class _GroupBN:
    """The seperate convs' three BatchNorms (plus `pad` identity channels) as ONE fused BN
    + ReLU launch.  Each of weight, bias, running_mean, running_var is concatenated with its
    cached constant identity padding by one cat (autograd routes the affine gradients back
    through the cat), the updated running statistics go back to the modules by one
    multi-tensor copy and num_batches_tracked advances by one multi-tensor add: 6 launches
    around the BN instead of ~20 (the modules' own buffers are left in place, so state_dict,
    .to() and the data-parallel buffer broadcast see ordinary buffers)."""

    def __init__(self):
        self.pads = {}

    def _pad(self, n, dev):
        p = self.pads.get((n, dev))
        if p is None:
            p = self.pads[(n, dev)] = (torch.ones(n, device=dev), torch.zeros(n, device=dev))
        return p

    def params(self, bns, pad, dev):
        """(weight, bias, running_mean, running_var) of the grouped BN: the modules' tensors
        concatenated with the identity padding."""
        ones, zeros = self._pad(pad, dev) if pad else (None, None)
        ext = (lambda ts, c: ts + [c]) if pad else (lambda ts, c: ts)
        return (torch.cat(ext([b.weight for b in bns], ones)), torch.cat(ext([b.bias for b in bns], zeros)),
                torch.cat(ext([b.running_mean for b in bns], zeros)), torch.cat(ext([b.running_var for b in bns], ones)))

    def __call__(self, x, bns, training, pad=0, levels=1, partials=None, cat=None):
        w, bi, rm, rv = cat if cat is not None else self.params(bns, pad, x.device)
        b0 = bns[0]
        y = ewvit.batch_norm_act_params(x, w, bi, rm, rv, training, b0.momentum, b0.eps, 'relu',
                                        levels if training else 1, partials=partials if training else None)
        if training:
            self.writeback(bns, rm, rv, levels)
        return y

    @staticmethod
    def writeback(bns, rm, rv, levels):
        """The grouped running statistics back into the modules; their counters += levels."""
        dst, src, off = [], [], 0
        for b in bns:
            n = b.num_features
            dst += [b.running_mean, b.running_var]
            src += [rm[off:off + n], rv[off:off + n]]
            off += n
        torch._foreach_copy_(dst, src)
        torch._foreach_add_([b.num_batches_tracked for b in bns], levels)


def bn_relu_groups(x, bns, training, pad=0, levels=1, state=None, partials=None, cat=None):
    """One fused BN + ReLU over the channel groups of `bns` (see _GroupBN); `state` keeps the
    grouped buffers between calls; `partials` (training): the batch statistics summed by the
    producing conv, with `cat` the grouped parameters the conv centred them on."""
    return (state if state is not None else _GroupBN())(x, bns, training, pad, levels, partials, cat)


def _cdt():
    return torch.get_autocast_dtype('cuda') if torch.is_autocast_enabled('cuda') else torch.float32


# tests compare the fused seperate conv + BN node against the two-node path
_FUSED_SEP_BN = True


class MWT(nn.Module):
    """Multi-level Wavelet Transformer (reference mwt.py:7-119)."""

    def __init__(self, in_channels=3, dama_dim=128, levels=3):
        super().__init__()
        self.in_channels = in_channels
        self.dama_dim = dama_dim
        self.levels = levels
        self.dwt = DWTForward(J=1, wave='haar', mode='zero')                  # mwt.py:20
        self.freq_conv = _cbr(dama_dim, dama_dim, stride=2)                    # mwt.py:23-36
        self.freq_pool = FreqPool(nn.MaxPool2d(kernel_size=2, stride=2),       # mwt.py:38-44
                                  Conv3x3(dama_dim, dama_dim, 3, padding=1, stride=2),
                                  nn.BatchNorm2d(dama_dim), nn.ReLU(inplace=True),
                                  nn.AdaptiveAvgPool2d(1))
        self.hf_conv = nn.ModuleDict({                                         # mwt.py:47-65
            'seperate': nn.ModuleList([_cbr(in_channels, 6 * in_channels, conv=nn.Conv2d) for _ in range(3)]),
            'fusion': _cbr(18 * in_channels, dama_dim)})
        self.multiscale_fusion = _cbr(levels * dama_dim, dama_dim)             # mwt.py:68-72

    # ---- reference API (mwt.py:74-90), one level
    def wavelet_transform(self, x, target_size):
        B, C, H, W = x.shape
        if self.levels > 1:
            hf, ll = ewvit.dwt_hf_upsample(x, 1, tuple(target_size), out_dtype=x.dtype if x.dtype == torch.bfloat16 else torch.float32,
                                           band_dtype=torch.float32)
            hf = hf[0].permute(0, 3, 1, 2)
        else:
            ll, yh = self.dwt(x)
            hf = yh[0].reshape(B, 3 * C, H // 2, W // 2)
        processed = [self.hf_conv['seperate'][i](hf[:, i * C:(i + 1) * C]) for i in range(3)]
        return ll, self.hf_conv['fusion'](torch.cat(processed, dim=1))

    def _patched(self):
        return 'wavelet_transform' in self.__dict__ or type(self).wavelet_transform is not MWT.wavelet_transform

    @bf16_compute
    def forward(self, x):
        B, C, H, W = x.shape
        target = (H // 2, W // 2)
        if self._patched():
            cur, highs = x, []
            for _ in range(self.levels):
                ll, hf = self.wavelet_transform(cur, target)
                highs.append(hf)
                cur = ll
            fused = self.multiscale_fusion(torch.cat(highs, dim=1))
            return self.freq_pool(self.freq_conv(fused))
        return self.freq_pool(self.freq_conv(self.multiscale_fusion(self._hf_features(x), self.levels)))

    def _hf_features(self, x):
        """All levels' hf_compressed, level-major [L*B, dim, H/2, W/2]; multiscale_fusion
        consumes it as the channel concatenation of mwt.py:112 (CBR(levels=L))."""
        B, C, H, W = x.shape
        Lv = self.levels
        OH, OW = H // 2, W // 2
        cdt = _cdt()
        out_hw = (OH, OW) if Lv > 1 else ((H + 1) // 2, (W + 1) // 2)
        # bf16: the 3C band channels zero-padded to a multiple of 16 in the same pass, so
        # the seperate conv runs on the ewvit MFMA conv (K = 9 taps x 16 channels)
        cin = 3 * C
        cpad = (cin + 15) // 16 * 16 if cdt == torch.bfloat16 else cin
        sep = self.hf_conv['seperate']
        convs = [sep[i][0] for i in range(3)]
        if (cdt == torch.bfloat16 and C == 3 and ewvit.hfsep.HF9 and x.is_cuda and out_hw[1] % 2 == 0
                and ewvit.hfsep.convs_apply(out_hw[1], convs)):
            cpad = 9        # the 9 real band channels: the hfsep kernels zero-pad K in LDS
        hf = ewvit.dwt_hf_features(x, Lv, out_hw, out_dtype=cdt, out_channels=cpad)
        hf = hf.view(Lv * B, out_hw[0], out_hw[1], cpad).permute(0, 3, 1, 2)   # NCHW view, NHWC memory
        if not hasattr(self, '_sep_bn'):
            self._sep_bn = _GroupBN()
        c18 = 18 * C
        pad = (-c18) % 64
        if C == 3 and cpad in (16, 9) and ewvit.hfsep.applies(hf, convs):
            # the grouped conv on csrc/hfsep.hip: 3 x (3 -> 18) for all levels in one launch,
            # 54 channels + 10 zero channels out (whole 64-channel K slices for the fusion
            # conv), the BatchNorm statistics per level summed on the way (training)
            bns = [sep[i][1] for i in range(3)]
            cat = self._sep_bn.params(bns, pad, hf.device)
            if self.training and pad == 10 and _FUSED_SEP_BN:
                # conv + BN + ReLU as one autograd node: its backward recomputes the BN's dx
                # inside the weight-gradient pass (ewvit.hfsep.SeperateBNReLUFn)
                y = ewvit.hfsep.seperate_conv_bn_relu(hf, Lv, convs, cat, bns[0].momentum, bns[0].eps)
                self._sep_bn.writeback(bns, cat[2], cat[3], Lv)
                return self._fusion(y, Lv, B)
            if self.training:
                y, partials = ewvit.hfsep.seperate_conv(hf, Lv, convs, shift=cat[2])
            else:
                y, partials = ewvit.hfsep.seperate_conv(hf, Lv, convs), None
            y = bn_relu_groups(y, bns, self.training, pad, Lv, self._sep_bn, partials, cat)
            return self._fusion(y, Lv, B)
        # seperate[i] sees colour i's 3C/3 = C band channels: a groups=3 conv.  It is
        # issued as ONE dense conv with a block-diagonal weight (zeros contribute
        # exact zeros): MIOpen's grouped weight-gradient kernel took ~0.3 s here.
        w = torch.cat([F.pad(sep[i][0].weight, (0, 0, 0, 0, i * C, (2 - i) * C + cpad - cin)) for i in range(3)])
        b = torch.cat([sep[i][0].bias for i in range(3)])
        # the fusion conv's MFMA kernels want 8-aligned channels, and its LDS-DMA
        # kernel whole 64-channel K-tiles: emit the 18C seperate channels zero-padded
        # to a multiple of 64 (zero weight rows and bias; an identity BN keeps them
        # exactly 0 through BN + ReLU, and the fusion weight's padded rows are zero)
        if pad:
            w = F.pad(w, (0, 0, 0, 0, 0, 0, 0, pad))
            b = F.pad(b, (0, pad))
        if cpad % 8 == 0 and hf.is_cuda:
            y = ewvit.conv2d(hf, w, b, 1)
        else:
            y = F.conv2d(hf, w.to(hf.dtype), b.to(hf.dtype), padding=1)
        # BN + ReLU of all levels in one fused launch, per-level statistics
        y = bn_relu_groups(y, [sep[i][1] for i in range(3)], self.training, pad, Lv, self._sep_bn)
        return self._fusion(y, Lv, B)

    def _fusion(self, y, Lv, B):
        """hf_conv['fusion'] (mwt.py:60-65, 87-88) over all levels, per-level BN statistics."""
        fus = self.hf_conv['fusion']
        r = _epi_stats(fus[0], fus[1], y, groups=Lv)
        if r is not None:
            ms = self.multiscale_fusion
            if (_FOLD_FUSION_BN and Lv > 1 and fus[1].track_running_stats and fus[1].momentum is not None
                    and not (fus[2]._forward_hooks or fus[2]._forward_pre_hooks or ms._forward_hooks
                             or ms._forward_pre_hooks)):
                # consumed by multiscale_fusion (CBR.forward), which applies BN + ReLU itself
                return PendingBNReLU(r[0], r[1], fus, Lv)
            return ewvit.batch_norm_act(r[0], fus[1], 'relu', groups=Lv, partials=r[1])
        z = fus[0](y)
        z = ewvit.batch_norm_act(z, fus[1], 'relu', groups=Lv) if _fusable(fus[1], z) else \
            torch.cat([fus[2](fus[1](z[l * B:(l + 1) * B])) for l in range(Lv)])
        return z
