"""ctypes binding of libewvit.so (the C-ABI declared in include/ewvit.h).

The library is built in-tree (``make -C csrc`` or ``__graft_entry__.build()``)
and loaded from this directory.  There is no fallback: if the library or a GPU
is missing, every op raises.
"""
import contextlib
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# EWVIT_LIB: another build of the library (A/B measurements of two kernel versions)
LIB_PATH = os.environ.get('EWVIT_LIB') or os.path.join(_HERE, 'libewvit.so')
ABI_VERSION = 3
F32, BF16 = 0, 1
ADAM_MAX = 48          # EWVIT_ADAM_MAX (include/ewvit.h)
PACK_MAX = 32          # EWVIT_PACK_MAX
ADAM_ENTRY = 7         # EWVIT_ADAM_ENTRY

_i64, _i32, _f32, _u64, _vp = ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p
_f64 = ctypes.c_double

# name -> argtypes (restype int for all but the two bookkeeping calls)
SIGNATURES = {
    'ewvit_dwt_haar_fwd': [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp],
    'ewvit_hf_upsample': [_vp, _vp, _i64, _i64, _i64, _i64, _i32, _i64, _i64, _i32, _i32, _i64, _vp],
    'ewvit_dwt_hf_upsample_fused': [_vp, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _i64, _vp],
    'ewvit_gemm': [_vp, _i32, _i64, _i64, _vp, _i32, _i64, _i64, _vp, _i32, _i64, _i64, _i64, _i64,
                   _f32, _f32, _vp, _i32, _vp, _f32, _u64, _vp, _vp, _i32, _i64, _i32, _vp, _vp],
    'ewvit_gemm_mx8': [_vp, _i32, _i64, _i64, _vp, _i32, _i64, _i64, _vp, _i32, _i64, _i64, _i64, _i64,
                       _f32, _f32, _vp, _i32, _vp, _f32, _u64, _vp, _vp, _i32, _i64, _i32, _vp, _vp],
    'ewvit_colsum': [_vp, _i32, _i64, _i64, _i64, _vp, _i32, _vp],
    'ewvit_dropout_bwd': [_vp, _i32, _i64, _i64, _i64, _f32, _u64, _vp, _vp],
    'ewvit_act_bwd': [_vp, _i32, _i64, _vp, _i32, _f32, _u64, _vp, _vp, _i32, _i64, _i64, _vp],
    'ewvit_layernorm_fwd': [_vp, _i32, _i64, _vp, _vp, _vp, _i32, _vp, _vp, _i64, _i64, _f32, _vp],
    'ewvit_layernorm_bwd': [_vp, _i32, _vp, _i32, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i64,
                            _i64, _vp],
    'ewvit_attn_fwd': [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64,
                       _i64, _i32, _i32, _i32, _f32, _vp],
    'ewvit_dwconv3x3_fwd': [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp],
    'ewvit_dwconv3x3_bwd_data': [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp],
    'ewvit_dwconv3x3_bwd_weight': [_vp, _vp, _vp, _i32, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp, _vp],
    'ewvit_bn_fwd': [_vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _i32, _f32, _f32, _i32, _vp, _vp, _i32, _vp,
                     _vp, _vp],
    'ewvit_bn_bwd': [_vp, _vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _vp, _vp],
    'ewvit_maxpool2_fwd': [_vp, _vp, _vp, _i32, _i64, _i64, _i64, _i64, _vp],
    'ewvit_maxpool2_bwd': [_vp, _vp, _vp, _i32, _i64, _i64, _i64, _i64, _vp],
    'ewvit_adam_step': [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _f64, _vp, _f64, _f64, _f32, _f32, _vp],
    'ewvit_conv2d_set_glds': [_i32],
    'ewvit_conv2d_set_win': [_i32],
    'ewvit_conv2d_set_lds_pad': [_i32],
    'ewvit_conv2d_set_wgrad_tap_split': [_i32],
    'ewvit_conv2d_set_win_nt': [_i32],
    'ewvit_dwt_set_pf': [_i32],
    'ewvit_conv2d_set_grid_cap': [_i32],
    'ewvit_set_grid_cap': [_i32],
    'ewvit_probe': [_vp, _i32, _vp],
    'ewvit_conv2d_set_wgrad_wide': [_i32],
    'ewvit_conv2d_set_wgrad_1x1': [_i32, _i32, _i32],
    'ewvit_conv2d_set_small_tiles': [_i32],
    'ewvit_conv2d_set_ksplit': [_i32],
    'ewvit_reduce_defer_next': [_i32],
    'ewvit_reduce_flush': [_vp],
    'ewvit_conv2d_pack_weights': [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    'ewvit_conv2d_pack_weight': [_vp, _i64, _i64, _i64, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
    'ewvit_conv2d_fwd_bn': [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i64, _i64, _vp, _vp,
                            _vp, _vp],
    'ewvit_conv2d_xf_ok': [_i64, _i64, _i64, _i64, _i64, _i32, _i32, _i64, _i64],
    'ewvit_conv2d_fwd_bn_xf': [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp,
                               _vp],
    'ewvit_conv2d_bwd_weight_xf': [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64,
                                   _i64, _i64, _i64, _vp, _vp],
    'ewvit_conv2d_bwd_data_bn_win': [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                                     _i32, _i64, _vp, _vp],
    'ewvit_bn_coef': [_i64, _i64, _vp, _vp, _vp, _vp, _f32, _f32, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp],
    'ewvit_bn_fwd_partials': [_vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _f32, _f32, _i32, _vp, _vp, _vp,
                              _vp, _vp, _i32, _i32, _vp],
    'ewvit_bn_fwd_drop_add': [_vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _f32, _f32, _vp, _vp, _vp, _vp, _vp,
                              _i32, _vp, _i64, _f32, _u64, _vp, _vp, _vp, _vp],
    'ewvit_bn_bwd_scaled': [_vp, _vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp],
    'ewvit_bn_bwd_se': [_vp, _vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _vp],
    'ewvit_bn_se_bwd': [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp,
                        _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    'ewvit_bn_se_bwd_dx': [_vp, _vp, _vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp],
    'ewvit_dwconv3x3_bwd_fused_se': [_vp, _vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                                     _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp],
    'ewvit_bn_fold_partials': [_vp, _i32, _vp, _vp, _i32, _vp, _i64, _i32, _vp],
    'ewvit_conv2d_fwd': [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i64, _i64, _vp],
    'ewvit_conv2d_stem_fwd': [_vp, _i32, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i32, _vp, _i64,
                              _i32, _vp, _vp, _vp, _vp],
    'ewvit_conv2d_bwd_data_add': [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _vp],
    'ewvit_conv2d_bwd_data': [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i64, _i64, _vp],
    'ewvit_conv2d_bwd_weight': [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i64, _i64,
                                _i64, _i64, _i64, _i64, _vp, _vp],
    'ewvit_se_reduce': [_vp, _vp, _i32, _i64, _i64, _i64, _f32, _vp, _vp, _vp],
    'ewvit_se_scale': [_vp, _i32, _vp, _vp, _vp, _i64, _i64, _i64, _vp],
    'ewvit_se_mlp_fwd': [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp],
    'ewvit_se_mlp_bwd': [_vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp],
    'ewvit_se_squeeze_mlp_fwd': [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp],
    'ewvit_se_squeeze_mlp_bwd': [_vp, _vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                                 _vp, _vp, _vp],
    'ewvit_scale_add': [_vp, _vp, _i32, _vp, _vp, _i64, _i64, _vp],
    'ewvit_scale_add_drop': [_vp, _vp, _i32, _f32, _u64, _vp, _vp, _vp, _i64, _i64, _vp],
    'ewvit_attn_bwd': [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _vp,
                       _vp, _vp, _i64, _i64, _i32, _i32, _i32, _f32, _vp],
    'ewvit_frames_resize_crop': [_vp, _vp, _i64, _i32, _vp, _i32, _vp, _vp, _vp],
    'ewvit_frames_jitter_normalize': [_vp, _vp, _i64, _i32, _vp, _vp, _vp],
    'ewvit_combined_loss': [_vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp],
    'ewvit_adam_step_table': [_vp, _i32, _i64, _f64, _vp, _f64, _f64, _f32, _f32, _vp],
    'ewvit_hfsep_fwd': [_vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    'ewvit_hfsep_bwd_weight': [_vp, _vp, _i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    'ewvit_bn_bwd_reduce': [_vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp],
    'ewvit_hfsep_bn_bwd_weight': [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp,
                                  _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    'ewvit_bn_act_se_squeeze': [_vp, _vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _f32, _f32, _i32, _vp, _vp,
                                _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _vp],
    'ewvit_se_gate_excite': [_vp, _vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    'ewvit_se_forward': [_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
    'ewvit_dwconv3x3_fwd_bn': [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp],
    'ewvit_dwconv3x3_bwd_data_bn': [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i32, _vp,
                                    _vp],
    'ewvit_dwconv3x3_bwd_fused': [_vp, _vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                                  _i32, _vp, _vp, _vp],
    'ewvit_bn_bwd_partials': [_vp, _vp, _vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i64, _vp,
                              _i32, _i32, _vp],
    'ewvit_head_fwd': [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp],
    'ewvit_head_bwd': [_vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64,
                       _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    'ewvit_conv2d_bwd_data_bn': [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i64, _i64, _vp, _vp,
                                 _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _vp],
    'ewvit_vit_layer_fwd': [_vp, _i32, _vp, _vp, _vp, _vp],
    'ewvit_vit_layer_bwd': [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    'ewvit_vit_pack': [_vp, _i32, _vp, _vp],
    'ewvit_vit_pack_mx': [_vp, _i32, _vp, _vp],
    'ewvit_gemm_tallk': [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp],
    'ewvit_vit_embed_fwd': [_vp, _vp, _vp, _i32, _i32, _f32, _u64, _vp, _vp, _vp],
    'ewvit_vit_embed_bwd': [_vp, _i32, _i32, _f32, _u64, _vp, _vp, _vp, _vp, _vp],
}

# size queries: name -> (restype, argtypes)
QUERIES = {
    'ewvit_conv2d_bwd_bn_win_rows': (_i64, [_i64, _i64, _i64, _i64, _i64, _i32, _i32, _i64, _i64, _i64]),
    'ewvit_layernorm_bwd_workspace': (_i64, [_i64, _i64]),
    'ewvit_vit_layer_workspace': (_i64, [_i32]),
    'ewvit_gemm_tallk_workspace': (_i64, [_i64, _i64, _i64]),
    'ewvit_dwconv3x3_bwd_weight_workspace': (_i64, [_i64, _i64, _i64, _i64, _i32, _i32]),
    'ewvit_dwconv3x3_bwd_fused_workspace': (_i64, [_i64, _i64, _i64, _i64]),
    'ewvit_conv2d_bwd_weight_workspace': (_i64, [_i64, _i64, _i64, _i64, _i64, _i32, _i32]),
    'ewvit_conv2d_fwd_bn_rows': (_i64, [_i64, _i64, _i64, _i64, _i64, _i32, _i32]),
    'ewvit_conv2d_stem_parts': (_i64, [_i64, _i64, _i64, _i32]),
    'ewvit_dwt_hf_fused_ok': (_i32, [_i64, _i64, _i64, _i64, _i32, _i64, _i64, _i64]),
    'ewvit_conv2d_fwd_pack_cin': (_i64, [_i64, _i64, _i64, _i64, _i64, _i32, _i32]),
    'ewvit_conv2d_bwd_data_add_ok': (_i64, [_i64, _i64, _i64, _i64, _i64, _i32, _i32]),
    'ewvit_bn_workspace': (_i64, [_i64, _i64, _i32]),
    'ewvit_se_reduce_workspace': (_i64, [_i64, _i64, _i64]),
    'ewvit_se_mlp_bwd_workspace': (_i64, [_i64, _i64, _i64]),
    'ewvit_bn_se_bwd_workspace': (_i64, [_i64, _i64, _i64]),
    'ewvit_bn_se_bwd_row_offset': (_i64, [_i64, _i64, _i64]),
    'ewvit_se_mlp_fwd_workspace': (_i64, [_i64, _i64, _i64]),
    'ewvit_frames_plan': (_i32, [_vp, _i64, _i32, _i64, _vp]),
    'ewvit_adam_chunks': (_i64, [_i64]),
    'ewvit_hfsep_fwd_parts': (_i64, [_i64, _i64, _i64, _i64]),
    'ewvit_hfsep_bwd_weight_workspace': (_i64, [_i64, _i64, _i64]),
    'ewvit_hfsep_bn_bwd_weight_workspace': (_i64, [_i64, _i64, _i64, _i64]),
    'ewvit_bn_bwd_reduce_rows': (_i32, [_i64, _i64, _i32]),
    'ewvit_dwconv3x3_bn_rows': (_i64, [_i64, _i64, _i64, _i64, _i32, _i32]),
    'ewvit_head_workspace': (_i64, []),
    'ewvit_head_pack_bytes': (_i64, []),
    'ewvit_head_pack_bytes_mx': (_i64, []),
    'ewvit_conv2d_bwd_bn_rows': (_i64, [_i64, _i64, _i64, _i64, _i64, _i32, _i32]),
    'ewvit_wall_clock_khz': (_i32, []),
    'ewvit_conv2d_wgrad_1x1_config': (_i32, [_i32]),
    'ewvit_reduce_pending': (_i32, [_vp]),
}

_lib = None


def load():
    """Load and type the library; raises RuntimeError when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f'ewvit: {LIB_PATH} not built — run `make -C csrc` '
                           '(or __graft_entry__.build()); there is no CPU fallback')
    lib = ctypes.CDLL(LIB_PATH)
    lib.ewvit_abi_version.restype = ctypes.c_int
    lib.ewvit_abi_version.argtypes = []
    lib.ewvit_last_error.restype = ctypes.c_char_p
    lib.ewvit_last_error.argtypes = []
    if lib.ewvit_abi_version() != ABI_VERSION:
        raise RuntimeError(f'ewvit: ABI {lib.ewvit_abi_version()} != expected {ABI_VERSION}')
    # (an EWVIT_LIB build for an A/B may predate entry points: those stay unbound)
    ab = bool(os.environ.get('EWVIT_LIB'))
    for name, args in SIGNATURES.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    for name, (res, args) in QUERIES.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if os.environ.get('EWVIT_SMALL_TILES') == '0' and hasattr(lib, 'ewvit_conv2d_set_small_tiles'):
        lib.ewvit_conv2d_set_small_tiles(0)          # A/B switch (conv.hip glds_tile)
    if os.environ.get('EWVIT_CONV_KSPLIT') and hasattr(lib, 'ewvit_conv2d_set_ksplit'):
        lib.ewvit_conv2d_set_ksplit(int(os.environ['EWVIT_CONV_KSPLIT']))   # A/B (conv.hip split K)
    if os.environ.get('EWVIT_LDS_PAD') == '0' and hasattr(lib, 'ewvit_conv2d_set_lds_pad'):
        lib.ewvit_conv2d_set_lds_pad(0)              # A/B switch (convwin.hip lds_pad)
    if os.environ.get('EWVIT_WGWIN_TS') in ('0', '2') and hasattr(lib, 'ewvit_conv2d_set_wgrad_tap_split'):
        lib.ewvit_conv2d_set_wgrad_tap_split(int(os.environ['EWVIT_WGWIN_TS']))   # A/B (convwin.hip wgrad NG)
    if os.environ.get('EWVIT_WIN_NT', '').isdigit() and hasattr(lib, 'ewvit_conv2d_set_win_nt'):
        lib.ewvit_conv2d_set_win_nt(int(os.environ['EWVIT_WIN_NT']))   # A/B switch (convwin.hip g_win_nt)
    if os.environ.get('EWVIT_WGRAD_WIDE') in ('0', '2') and hasattr(lib, 'ewvit_conv2d_set_wgrad_wide'):
        lib.ewvit_conv2d_set_wgrad_wide(int(os.environ['EWVIT_WGRAD_WIDE']))   # A/B (conv.hip wgrad_wide)
    if os.environ.get('EWVIT_W1X1') and hasattr(lib, 'ewvit_conv2d_set_wgrad_1x1'):
        # A/B: the 1x1 weight gradient's split rule "workgroup target:min K-tiles per split[:ring]"
        v = [int(x) for x in os.environ['EWVIT_W1X1'].split(':')]
        lib.ewvit_conv2d_set_wgrad_1x1(v[0], v[1], v[2] if len(v) > 2 else 0)
    if os.environ.get('EWVIT_DWTF_PF') in ('2', '4') and hasattr(lib, 'ewvit_dwt_set_pf'):
        lib.ewvit_dwt_set_pf(int(os.environ['EWVIT_DWTF_PF']))   # A/B switch (dwt.hip)
    _lib = lib
    return lib


# Optional per-launch timing (bench.py): HIP events recorded on the current stream
# — the stream every ewvit kernel is launched on — around each launch, with the
# launch's algorithmic work (bytes, flops) attached.
_timers = None


def enable_timing(on=True):
    global _timers
    _timers = {} if on else None


def timing_records():
    return _timers or {}


def timing_detail():
    """[(entry, integer args, start event, end event)] in launch order (layer attribution)."""
    return (_timers or {}).get('__detail__', [])


def call(name, *args, work=None):
    rec = _timers is not None
    if rec:
        s = torch.cuda.Event(enable_timing=True)
        s.record()
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f'{name} failed (rc={rc}): {_lib.ewvit_last_error().decode()}')
    if rec:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        _timers.setdefault(name, []).append((s, e, work or {}))
        ints = tuple(a for a in args if isinstance(a, int) and not isinstance(a, bool))
        _timers.setdefault('__detail__', []).append((name, ints, s, e, work or {}))


def dt(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f'ewvit: unsupported dtype {t.dtype} (f32/bf16 only)')


_rng_offsets = {}


def rng_offset(device):
    """Device int64 step counter mixed into every dropout seed (csrc/common.h
    step_seed): a launch recorded in a HIP graph reads it on each replay, so a
    replayed step draws fresh masks once the counter is advanced."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = _rng_offsets.get(idx)
    if t is None:
        t = torch.zeros(1, dtype=torch.int64, device=torch.device('cuda', idx))
        _rng_offsets[idx] = t
    return t


def rng_advance(device):
    """Advance the dropout step counter (a device op: recorded into a captured step)."""
    rng_offset(device).add_(1)


# Workgroup cap of the big-grid launches (LDS-DMA convs, BatchNorm passes) while
# `grid_cap(n)` is active: a branch that runs on its own stream beside another (DAMA's MWT
# beside the backbone) walks its tiles / rows on part of the CUs instead of filling the whole
# GPU.  Ops remember the cap of their forward for their backward launches (`launch_cap`).
# Per thread, like the C side (ewvit_set_grid_cap): nn.DataParallel runs its replicas in
# threads (reference train.py:249-251), and one replica's branch cap must not leak into another.
_tls = threading.local()


@contextlib.contextmanager
def grid_cap(n):
    prev = getattr(_tls, 'cap', 0)
    _tls.cap = int(n)
    try:
        yield
    finally:
        _tls.cap = prev


# the backward's cap for ops whose forward ran capped (EWVIT_MWT_BWD_CAP, A/B; unset: the same cap)
_BWD_CAP = int(os.environ.get('EWVIT_MWT_BWD_CAP', '0') or 0)


def bwd_cap(n):
    """The cap for the backward of an op whose forward ran under cap n: the same (one cap
    balances both phases), or EWVIT_MWT_BWD_CAP when set."""
    return _BWD_CAP if (n and _BWD_CAP > 0) else n


def has(name):
    """The loaded library exports `name` (an older EWVIT_LIB build for an A/B may not: the
    callers of entry points added within an ABI version fall back to the older path)."""
    return hasattr(load(), name)


def current_cap():
    return getattr(_tls, 'cap', 0)


@contextlib.contextmanager
def launch_cap(n):
    """The C-side cap for the launches issued inside (ewvit_set_grid_cap)."""
    if not n:
        yield
        return
    prev = load().ewvit_set_grid_cap(int(n))
    try:
        yield
    finally:
        load().ewvit_set_grid_cap(prev)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError('ewvit ops run on the MI355X only (tensor on %s); the product has no '
                               'CPU path — use the oracle for CPU reference numbers' % t.device)
