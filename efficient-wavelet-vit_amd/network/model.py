"""DeepfakeDetector — drop-in for reference network/model.py:9-171 ('dynamic' mode).

The reference also constructs ``mwt``, ``sfe``, ``sfe_cls`` (EfficientNet-b0 via
``efficientnet_pytorch.from_pretrained``, a network fetch) and ``fusion_gate``
for the 'sfe_only' / 'sfe_mwt' ablations (model.py:37-58,100-161).  Those heads
are outside the hot path (SURVEY §2 OUT rows); ``mwt``, ``fusion_gate`` and
``feat_pooler`` are built for state-dict compatibility, the b0 heads are not built up
front.  ``load_state_dict`` accepts reference checkpoints unchanged — so the reference's
``eval.py:60-77`` (strict ``model.load_state_dict(torch.load(path))``) works as is: the
DataParallel ``module.`` prefix (train.py:309,315) is stripped, and every ``sfe.*`` /
``sfe_cls.*`` tensor of the b0 heads is kept in a parameter-free placeholder under the
same key, so it loads strictly and is saved back by ``state_dict()`` (round trip), while
no compute ever touches it.
"""
from collections import OrderedDict

import torch
from torch import nn

import ewvit

from . import bf16_compute, load_config
from .dama import DAMA
from .mwt import MWT
from .sfe import Linear, _hooked


class DeepfakeDetector(nn.Module):
    def __init__(self, in_channels=3, dama_dim=128, batch_size=16, ablation='dynamic'):
        super().__init__()
        self.dama_dim = dama_dim
        self.in_channels = in_channels
        self.batch_size = batch_size
        self.ablation_config = ['dynamic', 'sfe_only', 'sfe_mwt']
        self.ablation = ablation
        self.config = load_config()
        self.dama = DAMA(in_channels=in_channels, dim=dama_dim, num_heads=4, levels=3, batch_size=batch_size)
        self.mwt = MWT(in_channels=in_channels, dama_dim=dama_dim)
        self.fusion_gate = nn.Sequential(nn.Linear(dama_dim * 2, 2), nn.ReLU(), nn.Dropout(0.1))
        self.feat_pooler = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(Linear(dama_dim, 64), nn.ReLU(), nn.Dropout(0.3), Linear(64, 1))
        # the ablation-only members are unused in 'dynamic' mode (SURVEY §8a note 5)
        # (and EfficientViT.mlp_head: output_mode='feature_map' never calls it, sfe.py:134-138,166)
        unused = list(self.mwt.parameters()) + list(self.fusion_gate.parameters()) + \
            list(self.dama.sfe.mlp_head.parameters())
        for p in unused:
            p.requires_grad_(False)

    def _classify(self, f):
        c = self.classifier
        if _hooked(c):
            return c(f)
        l1, drop, l2 = c[0], c[2], c[3]
        h = ewvit.linear(f, l1.weight, l1.bias, act=2, drop_p=drop.p if self.training else 0.0,
                         out_dtype=torch.float32)
        return ewvit.linear(h, l2.weight, l2.bias, out_dtype=torch.float32)

    @bf16_compute
    def forward(self, x, batch_size, ablation):
        if batch_size is not None:
            self.batch_size = batch_size
        if ablation is not None:
            self.ablation = ablation
        if self.ablation != 'dynamic':
            raise NotImplementedError(f"ablation '{self.ablation}' needs EfficientNet-b0 (network fetch); "
                                      "only 'dynamic' (the DAMA hot path) is provided")
        d = self.dama(x, batch_size=self.batch_size)
        return {'logits': self._classify(d['fused']), 'fused': d['fused'], 'space': d['space'],
                'freq': d['freq']}

    _ABLATION_HEADS = ('sfe', 'sfe_cls')

    def _hold_ablation_tensor(self, key, value):
        """Register `value`'s shape under `key` (e.g. sfe.efficient_net._fc.weight) in
        placeholder modules — buffers, not parameters: they never train."""
        parts = key.split('.')
        mod = self
        for name in parts[:-1]:
            child = mod._modules.get(name)
            if child is None:
                child = _AblationHeadState()
                mod.add_module(name, child)
            mod = child
        dev = self.classifier[0].weight.device
        if not isinstance(mod, _AblationHeadState):
            raise KeyError(f'{key}: not an ablation-head key')
        mod.register_buffer(parts[-1], torch.empty(value.shape, dtype=value.dtype, device=dev))

    def load_state_dict(self, state_dict, strict=True, assign=False):
        """nn.Module.load_state_dict accepting the reference's checkpoints (see module doc)."""
        sd = OrderedDict((k[7:] if k.startswith('module.') else k, v) for k, v in state_dict.items())
        for k, v in sd.items():
            if k.split('.', 1)[0] in self._ABLATION_HEADS and torch.is_tensor(v):
                self._hold_ablation_tensor(k, v)
        return super().load_state_dict(sd, strict=strict, assign=assign)

    def configure_ablation(self, ablation):
        if ablation in self.ablation_config:
            self.ablation = ablation
        else:
            raise ValueError(f'Invalid ablation config: {ablation}.')


class _AblationHeadState(nn.Module):
    """Holds checkpoint tensors of the reference's b0 ablation heads (model.py:37-51); no forward.

    Nothing trains or updates them, so the data-parallel buffer broadcast leaves them out
    (ewvit.graph.BufferSync: a resumed reference checkpoint would otherwise broadcast two
    128 MB patch_to_embedding weights every step)."""

    ewvit_buffer_sync = False

    def forward(self, *_):
        raise NotImplementedError("the 'sfe_only' / 'sfe_mwt' ablation heads need EfficientNet-b0 "
                                  "(a network fetch); only their checkpoint tensors are kept")


def load_reference_state_dict(model, state_dict):
    """Load a reference (possibly DataParallel-wrapped) checkpoint without the b0 ablation
    heads; returns the (missing, unexpected) key lists."""
    sd = {k[7:] if k.startswith('module.') else k: v for k, v in state_dict.items()}
    sd = {k: v for k, v in sd.items() if k.split('.', 1)[0] not in DeepfakeDetector._ABLATION_HEADS}
    res = nn.Module.load_state_dict(model, sd, strict=False)
    return res.missing_keys, res.unexpected_keys
