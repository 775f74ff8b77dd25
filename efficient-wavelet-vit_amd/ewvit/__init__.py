"""ewvit — MI355X (gfx950) kernels of the Efficient-Wavelet-ViT hot path.

C-ABI: include/ewvit.h, built into ewvit/libewvit.so from csrc/*.hip.
"""
from . import _lib, head, hfsep, optim, vit
from .bn import batch_norm_act, batch_norm_act_params, batch_norm_drop_add
from .conv import conv2d, conv3x3
from .se import bn_act_se, drop_add, scale_add, squeeze_excite
from .ops import (attention_cross, attention_packed, colsum, dwconv3x3, dwt_haar, dwt_hf_features, dwt_hf_upsample, gemm, maxpool2,
                  hf_upsample, layer_norm, linear, mm_nn, mm_nt, mm_tn)

__all__ = ['attention_cross', 'attention_packed', 'colsum', 'conv2d', 'conv3x3', 'dwconv3x3', 'dwt_haar', 'dwt_hf_features', 'dwt_hf_upsample', 'gemm',
           'hf_upsample', 'layer_norm', 'linear', 'maxpool2', 'mm_nn', 'mm_nt', 'mm_tn', 'bn_act_se', 'drop_add', 'scale_add', 'squeeze_excite',
           'load_library']


def load_library():
    return _lib.load()
