"""EfficientNetV2-S feature extractor — the spatial backbone DAMA builds through
``EfficientViT(selected_efficient_net=1)`` (reference network/sfe.py:111-113, there
``torchvision.models.efficientnet_v2_s``; torchvision is not part of this stack).

Module tree and parameter names follow torchvision's published model so
reference checkpoints load key-for-key (``features.{stage}.{block}.block.{i}...``).
Layout: the backbone runs channels-last (NHWC), which the ewvit conv / depthwise /
BatchNorm kernels and the ewvit head all want (the 7x7x1280 map is then already the
``(p1 p2 c)`` patch vector of sfe.py:153).

Stages (expand, kernel, stride, in, out, blocks): FusedMBConv (1,3,1,24,24,2)
(4,3,2,24,48,4) (4,3,2,48,64,4); MBConv (4,3,2,64,128,6) (6,3,1,128,160,9)
(6,3,2,160,256,15); stem 3x3 s2 3->24, head 1x1 256->1280; BN eps 1e-3; SiLU;
squeeze-excitation width = block input // 4; stochastic depth 0.2 * i / 40.
"""
import os

import torch
from torch import nn

import ewvit

# BatchNorm statistics summed in the producing conv's epilogue when the conv has at
# most this many 128-row output tiles: every BN apply block re-reads all partial rows
# while finalising, so the fusion pays only for small maps.  128 (the stage-5 14^2 maps at 64
# frames now included) after the deferred reductions: 3904-3916 against 3886-3890 frames/s at 32,
# 512 3874-3901, unbounded 3898-3899 (profiles/r06/s2/ab/epi_stats_tiles.log)
_EPI_STATS_MAX_TILES = int(os.environ.get('EWVIT_EPI_STATS_MAX_TILES', '128'))
# residual blocks hand their skip gradient to the first conv's dgrad epilogue (SkipLink)
_SKIP_LINK = os.environ.get('EWVIT_SKIP_LINK', '1') != '0'
# the frozen 3-channel stem on the ewvit direct conv (0: the library conv, A/B)
_STEM = os.environ.get('EWVIT_STEM', '1') != '0'
# MBConv's depthwise BN + SiLU and its squeeze-excitation as one ewvit.bn_act_se (0: A/B)
_BN_SE = os.environ.get('EWVIT_BN_SE', '1') != '0'
# the depthwise conv sums its BatchNorm's statistics (0: a statistics pass, A/B)
_DW_STATS = os.environ.get('EWVIT_DW_STATS', '1') != '0'

STAGES = (
    ('fused', 1, 3, 1, 24, 24, 2),
    ('fused', 4, 3, 2, 24, 48, 4),
    ('fused', 4, 3, 2, 48, 64, 4),
    ('mb', 4, 3, 2, 64, 128, 6),
    ('mb', 6, 3, 1, 128, 160, 9),
    ('mb', 6, 3, 2, 160, 256, 15),
)


def _divisible(v, d=8):
    n = max(d, int(v + d / 2) // d * d)
    return n + d if n < 0.9 * v else n


class DepthwiseConv2d(nn.Conv2d):
    """3x3 depthwise conv (groups = channels) on the ewvit channels-last kernels
    (csrc/depthwise.hip); parameters identical to nn.Conv2d."""

    def forward(self, x):
        return ewvit.dwconv3x3(x, self.weight, self.stride[0], self.padding[0])


class Conv2d(nn.Conv2d):
    """Dense 1x1 / 3x3 conv (padding k//2, no dilation, groups 1) on the ewvit MFMA
    implicit-GEMM kernels (csrc/conv.hip) when both channel counts are multiples
    of 8.  The 3-channel stem, frozen on the training path, runs the ewvit direct conv
    through ConvBNAct._stem; a stem that takes a gradient stays on the library conv.
    Parameters identical to nn.Conv2d."""

    def forward(self, x):
        k = self.kernel_size[0]
        if (x.is_cuda and k in (1, 3) and self.kernel_size[1] == k and self.groups == 1 and
                self.padding == (k // 2, k // 2) and self.dilation == (1, 1) and self.stride[0] == self.stride[1] and
                self.in_channels % 8 == 0 and self.out_channels % 8 == 0 and x.shape[1] == self.in_channels):
            return ewvit.conv2d(x, self.weight, self.bias, self.stride[0])
        return super().forward(x)


class ConvBNAct(nn.Sequential):
    """conv -> BatchNorm2d(eps 1e-3) [-> SiLU]; BN and SiLU run as ONE fused ewvit
    pass (csrc/batchnorm.hip) over the channels-last conv output."""

    def __init__(self, cin, cout, k, stride=1, groups=1, act=True):
        conv = DepthwiseConv2d if (groups == cin == cout and groups > 1 and k == 3) else Conv2d
        mods = [conv(cin, cout, k, stride, (k - 1) // 2, groups=groups, bias=False),
                nn.BatchNorm2d(cout, eps=1e-3)]
        if act:
            mods.append(nn.SiLU(inplace=True))
        super().__init__(*mods)

    def _hooked(self):
        return any(m._forward_hooks or m._forward_pre_hooks for m in self)

    def _conv_stats(self, x):
        """(y, partials) with the BatchNorm statistics summed in the conv's epilogue, or None."""
        conv, bn = self[0], self[1]
        if (type(conv) is Conv2d and bn.training and bn.track_running_stats and bn.momentum is not None
                and not self._hooked() and x.is_cuda and conv.groups == 1
                and conv.padding[0] == conv.kernel_size[0] // 2 and conv.stride[0] == conv.stride[1]
                and conv.out_channels <= 2048):
            rows = ewvit.conv.bn_stat_rows(x, conv.weight, conv.stride[0])
            # (counted in 128-row tiles whatever the kernel's row tile: 64 on small grids)
            if rows and (x.shape[0] * ((x.shape[2] - 1) // conv.stride[0] + 1) *
                         ((x.shape[3] - 1) // conv.stride[0] + 1) + 127) // 128 <= _EPI_STATS_MAX_TILES:
                r = ewvit.conv.conv2d_bn_stats(x, conv.weight, conv.bias, conv.stride[0], bn.running_mean)
                if r is not None:
                    return r[0], r[1:]
        return None

    def dw_stats(self, x, selink=None):
        """(y, part, shifts, nrc): the depthwise conv with its BatchNorm's statistics summed by
        the conv kernel (ewvit.ops.dwconv3x3_bn_stats), or None.  `selink`: the BN + SE after it
        may leave its backward's dx pass to the conv (ewvit.se.SeDxLink)."""
        conv, bn = self[0], self[1]
        if not (_DW_STATS and type(conv) is DepthwiseConv2d and conv.padding == (1, 1) and bn.training
                and bn.track_running_stats and bn.momentum is not None and x.is_cuda and not self._hooked()):
            return None
        return ewvit.ops.dwconv3x3_bn_stats(x, conv.weight, conv.stride[0], bn.running_mean, selink)

    def can_bn_se(self, x, se):
        """This block's BatchNorm + act on input x's conv output, then `se`, as one
        ewvit.bn_act_se."""
        bn, c = self[1], self[0].out_channels
        return (_BN_SE and bn.training and bn.track_running_stats and bn.momentum is not None and x.is_cuda
                and x.dim() == 4 and c % 8 == 0 and c <= 4096 and not self._hooked()
                and isinstance(se, SqueezeExcitation) and not se._has_hooks())

    def can_drop_add(self, x):
        bn = self[1]
        return (len(self) == 2 and type(self[0]) is Conv2d and bn.training and bn.momentum is not None
                and x.is_cuda and not self._hooked() and self[0].out_channels % 8 == 0
                and self[0].out_channels <= 4096)

    def forward_drop_add(self, x, skip, drop_prob, link=None):
        """StochasticDepth(bn(conv(x))) + skip: BN, drop-path and the skip add in one pass."""
        r = self._conv_stats(x)
        if r is not None:
            return ewvit.batch_norm_drop_add(r[0], self[1], skip, drop_prob, partials=r[1], link=link)
        return ewvit.batch_norm_drop_add(self[0](x), self[1], skip, drop_prob, link=link)

    def _stem(self, x, act):
        """The frozen 3-channel stem (sfe.py:115-119 freezes backbone parameters 0-5): the
        forward-only ewvit direct conv reading the fp32 NCHW frames, with the BatchNorm
        statistics summed on the way in training; None when it does not apply."""
        conv, bn = self[0], self[1]
        if not (type(conv) is Conv2d and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
                and conv.stride[0] == conv.stride[1] and not self._hooked()
                and ewvit.conv.stem_ok(x, conv.weight, conv.bias, conv.stride[0])):
            return None
        if bn.training and bn.track_running_stats and bn.momentum is not None:
            r = ewvit.conv.stem_conv2d(x, conv.weight, conv.bias, conv.stride[0], bn.running_mean, stats=True)
            return ewvit.batch_norm_act(r[0], bn, act, partials=r[1:])
        return ewvit.batch_norm_act(ewvit.conv.stem_conv2d(x, conv.weight, conv.bias, conv.stride[0]), bn, act)

    def forward(self, x):
        conv, bn = self[0], self[1]
        act = 'silu' if len(self) > 2 else None
        if _STEM and x.is_cuda and x.shape[1] <= 4:
            y = self._stem(x, act)
            if y is not None:
                return y
        r = self._conv_stats(x)
        if r is not None:
            # the conv's epilogue summed the batch statistics: BN runs its apply pass only
            return ewvit.batch_norm_act(r[0], bn, act, partials=r[1])
        y = conv(x)
        if y.is_cuda and y.shape[1] % 8 == 0 and y.shape[1] <= 2048 and not (bn._forward_hooks or bn._forward_pre_hooks):
            return ewvit.batch_norm_act(y, bn, act)
        y = bn(y)
        return self[2](y) if len(self) > 2 else y


class SqueezeExcitation(nn.Module):
    def __init__(self, cin, csq):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(cin, csq, 1)
        self.fc2 = nn.Conv2d(csq, cin, 1)
        self.activation = nn.SiLU(inplace=True)
        self.scale_activation = nn.Sigmoid()

    def forward(self, x):
        if x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0 and not self._has_hooks():
            return ewvit.squeeze_excite(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias)
        s = self.scale_activation(self.fc2(self.activation(self.fc1(self.avgpool(x)))))
        return x * s

    def _has_hooks(self):
        return any(m._forward_hooks or m._forward_pre_hooks for m in self.modules())


def _drop_path(x, p, training):
    """StochasticDepth(mode='row'): per-sample keep with prob 1-p, rescaled."""
    if not training or p == 0.0:
        return x
    keep = torch.empty((x.shape[0], 1, 1, 1), dtype=x.dtype, device=x.device).bernoulli_(1.0 - p)
    return x * keep.div_(1.0 - p)


def _seq(mods, h):
    """Run a block's modules in order; a depthwise ConvBNAct followed by its SqueezeExcitation
    runs as conv + ewvit.bn_act_se (the SE input-gradient pass folded into the BatchNorm
    backward)."""
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, ConvBNAct) and i + 1 < len(mods) and m.can_bn_se(h, mods[i + 1]):
            se = mods[i + 1]
            # the BN + SE backward's dx pass folded into the depthwise conv's backward (SeDxLink)
            link = ewvit.se.SeDxLink() if torch.is_grad_enabled() else None
            r = m.dw_stats(h, link)
            if r is None:
                link = None
            y, part = (r[0], r[1:]) if r is not None else (m[0](h), None)
            h = ewvit.bn_act_se(y, m[1], 'silu' if len(m) > 2 else None, se.fc1.weight, se.fc1.bias,
                                se.fc2.weight, se.fc2.bias, partials=part, link=link)
            i += 2
            continue
        h = m(h)
        i += 1
    return h


def r_ok(x):
    return x.dtype in (torch.bfloat16, torch.float32) and x.dim() == 4 and x.shape[1] % 8 == 0


class _Block(nn.Module):
    def forward(self, x):
        last = self.block[-1]
        if (self.use_res_connect and self.training and isinstance(last, ConvBNAct) and last.can_drop_add(x)
                and r_ok(x) and not self._forward_hooks and not self.block._forward_hooks):
            # the block tail (project BN + drop-path + skip add) as one pass each way; the
            # skip's gradient is added in the first conv's dgrad epilogue (SkipLink)
            link = ewvit.conv.offer_skip_link(x) if torch.is_grad_enabled() and _SKIP_LINK else None
            h = _seq(list(self.block)[:-1], x)
            ewvit.conv.clear_skip_link()
            return last.forward_drop_add(h, x, self.sd_prob, link)
        r = self.block(x) if self.block._forward_hooks or self.block._forward_pre_hooks else _seq(list(self.block), x)
        if self.use_res_connect:
            if self.training and self.sd_prob > 0.0 and r.is_cuda and r.dtype in (torch.bfloat16, torch.float32) \
                    and (r[0].numel() % 8 == 0):
                # StochasticDepth(row) + skip add in ONE pass, the keep mask drawn in the
                # kernel (counter-hash RNG like ewvit dropout: same distribution as
                # torchvision's bernoulli_, not its random stream)
                return ewvit.drop_add(r, x, self.sd_prob)
            return _drop_path(r, self.sd_prob, self.training) + x
        return r


class FusedMBConv(_Block):
    def __init__(self, expand, k, stride, cin, cout, sd_prob):
        super().__init__()
        mid = _divisible(cin * expand)
        self.use_res_connect = stride == 1 and cin == cout
        if mid != cin:
            self.block = nn.Sequential(ConvBNAct(cin, mid, k, stride), ConvBNAct(mid, cout, 1, act=False))
        else:
            self.block = nn.Sequential(ConvBNAct(cin, cout, k, stride))
        self.sd_prob = sd_prob


class MBConv(_Block):
    def __init__(self, expand, k, stride, cin, cout, sd_prob):
        super().__init__()
        mid = _divisible(cin * expand)
        self.use_res_connect = stride == 1 and cin == cout
        mods = [ConvBNAct(cin, mid, 1)] if mid != cin else []
        mods += [ConvBNAct(mid, mid, k, stride, groups=mid), SqueezeExcitation(mid, max(1, cin // 4)),
                 ConvBNAct(mid, cout, 1, act=False)]
        self.block = nn.Sequential(*mods)
        self.sd_prob = sd_prob


class EfficientNetV2S(nn.Module):
    def __init__(self, num_classes=1000, stochastic_depth_prob=0.2, dropout=0.2):
        super().__init__()
        layers = [ConvBNAct(3, 24, 3, 2)]
        total = sum(s[-1] for s in STAGES)
        i = 0
        for kind, e, k, st, cin, cout, n in STAGES:
            blk = FusedMBConv if kind == 'fused' else MBConv
            stage = []
            for j in range(n):
                stage.append(blk(e, k, st if j == 0 else 1, cin if j == 0 else cout, cout,
                                 stochastic_depth_prob * i / total))
                i += 1
            layers.append(nn.Sequential(*stage))
        layers.append(ConvBNAct(256, 1280, 1))
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(nn.Dropout(p=dropout, inplace=True), nn.Linear(1280, num_classes))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out')
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                r = 1.0 / (m.out_features ** 0.5)
                nn.init.uniform_(m.weight, -r, r)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = torch.flatten(self.avgpool(self.features(x)), 1)
        return self.classifier(x)


def efficientnet_v2_s(weights=None, **kw):
    if weights is not None:
        raise RuntimeError('EfficientNetV2-S IMAGENET1K_V1 weights need a network fetch; load a '
                           'state_dict instead')
    return EfficientNetV2S(**kw)
