"""ORACLE (test infrastructure only) — torch fp32 restatement of torchvision's
``efficientnet_v2_s`` (the backbone the reference builds at ``network/sfe.py:111-113``
and calls as ``self.efficient_net.features(img)`` at ``network/sfe.py:150``).

torchvision is absent from this image (and its IMAGENET1K_V1 weights are a
network fetch), so the published architecture is restated here with the same
module tree, so state-dict keys match torchvision's exactly
(``features.{i}.{j}.block.{k}...``):

* stem Conv3x3 s2 3->24 + BN(eps 1e-3) + SiLU
* FusedMBConv (expand, k, stride, in, out, layers):
  (1,3,1,24,24,2) (4,3,2,24,48,4) (4,3,2,48,64,4)
* MBConv: (4,3,2,64,128,6) (6,3,1,128,160,9) (6,3,2,160,256,15)
  with SqueezeExcitation(squeeze = in//4, SiLU, Sigmoid)
* head Conv1x1 256->1280 + BN + SiLU
* StochasticDepth("row") with p = 0.2 * block_id / 40 (train mode only)
* classifier = Dropout(0.2) + Linear(1280, 1000) (the reference replaces it by
  nn.Identity, sfe.py:114)

Parameter count with the 1000-class head: 21,458,488 (torchvision's published
number) — asserted in tests/test_oracle.py.
"""
import torch
from torch import nn


def make_divisible(v, divisor=8, min_value=None):
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def conv_norm_act(cin, cout, k, stride=1, groups=1, act=True):
    layers = [nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, groups=groups, bias=False),
              nn.BatchNorm2d(cout, eps=1e-3)]
    if act:
        layers.append(nn.SiLU(inplace=True))
    return nn.Sequential(*layers)


class SqueezeExcitation(nn.Module):
    def __init__(self, cin, csq):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(cin, csq, 1)
        self.fc2 = nn.Conv2d(csq, cin, 1)
        self.activation = nn.SiLU(inplace=True)
        self.scale_activation = nn.Sigmoid()

    def forward(self, x):
        s = self.scale_activation(self.fc2(self.activation(self.fc1(self.avgpool(x)))))
        return s * x


def stochastic_depth(x, p, training):
    if not training or p == 0.0:
        return x
    survival = 1.0 - p
    noise = torch.empty([x.shape[0], 1, 1, 1], dtype=x.dtype, device=x.device).bernoulli_(survival)
    if survival > 0.0:
        noise.div_(survival)
    return x * noise


class MBConv(nn.Module):
    def __init__(self, expand, k, stride, cin, cout, sd_prob):
        super().__init__()
        self.use_res_connect = stride == 1 and cin == cout
        mid = make_divisible(cin * expand)
        layers = []
        if mid != cin:
            layers.append(conv_norm_act(cin, mid, 1))
        layers.append(conv_norm_act(mid, mid, k, stride, groups=mid))
        layers.append(SqueezeExcitation(mid, max(1, cin // 4)))
        layers.append(conv_norm_act(mid, cout, 1, act=False))
        self.block = nn.Sequential(*layers)
        self.sd_prob = sd_prob

    def forward(self, x):
        r = self.block(x)
        if self.use_res_connect:
            r = stochastic_depth(r, self.sd_prob, self.training)
            r = r + x
        return r


class FusedMBConv(nn.Module):
    def __init__(self, expand, k, stride, cin, cout, sd_prob):
        super().__init__()
        self.use_res_connect = stride == 1 and cin == cout
        mid = make_divisible(cin * expand)
        if mid != cin:
            layers = [conv_norm_act(cin, mid, k, stride), conv_norm_act(mid, cout, 1, act=False)]
        else:
            layers = [conv_norm_act(cin, cout, k, stride)]
        self.block = nn.Sequential(*layers)
        self.sd_prob = sd_prob

    def forward(self, x):
        r = self.block(x)
        if self.use_res_connect:
            r = stochastic_depth(r, self.sd_prob, self.training)
            r = r + x
        return r


V2S_SETTING = [
    (FusedMBConv, 1, 3, 1, 24, 24, 2),
    (FusedMBConv, 4, 3, 2, 24, 48, 4),
    (FusedMBConv, 4, 3, 2, 48, 64, 4),
    (MBConv, 4, 3, 2, 64, 128, 6),
    (MBConv, 6, 3, 1, 128, 160, 9),
    (MBConv, 6, 3, 2, 160, 256, 15),
]


class EfficientNetV2S(nn.Module):
    def __init__(self, num_classes=1000, stochastic_depth_prob=0.2, dropout=0.2):
        super().__init__()
        layers = [conv_norm_act(3, 24, 3, 2)]
        total = sum(s[-1] for s in V2S_SETTING)
        bid = 0
        for blk, e, k, st, cin, cout, n in V2S_SETTING:
            stage = []
            for i in range(n):
                sd = stochastic_depth_prob * float(bid) / total
                stage.append(blk(e, k, st if i == 0 else 1, cin if i == 0 else cout, cout, sd))
                bid += 1
            layers.append(nn.Sequential(*stage))
        layers.append(conv_norm_act(256, 1280, 1))
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(nn.Dropout(p=dropout, inplace=True), nn.Linear(1280, num_classes))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
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
        x = self.features(x)
        x = torch.flatten(self.avgpool(x), 1)
        return self.classifier(x)


def efficientnet_v2_s(weights=None, **kw):
    """torchvision signature; ``weights`` must be None (no network here)."""
    if weights is not None:
        raise RuntimeError("pretrained EfficientNetV2-S weights are not reachable offline")
    return EfficientNetV2S(**kw)
