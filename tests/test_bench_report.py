"""bench.py's roofline reporting (host logic only, no GPU): each MFMA entry point is priced
against the dense peak of the dtype it computes in, HBM-bound entries against HBM3E."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _row(tfs, gbs):
    return {'TFLOP/s': tfs, 'GB/s': gbs, 'avg_us': 10.0, 'flops_per_launch': 1e9, 'bytes_per_launch': 1e6,
            'per_step': 1.0}


def test_fp8_gemm_priced_against_fp8_peak():
    import bench
    r = bench.roofline_for('ewvit_gemm_fp8', _row(500.0, 0.0), config=5)
    assert r['bound'] == 'mfma' and r['peak'] == bench.FP8_PEAK_TFS == 5000.0
    assert abs(r['frac'] - 0.1) < 1e-9


def test_bf16_gemm_and_conv_priced_against_bf16_peak():
    import bench
    for name in ('ewvit_gemm', 'ewvit_conv2d_bwd_weight'):
        r = bench.roofline_for(name, _row(250.0, 0.0))
        assert r['peak'] == bench.BF16_PEAK_TFS and abs(r['frac'] - 0.1) < 1e-9


def test_hbm_entry_priced_against_hbm():
    import bench
    r = bench.roofline_for('ewvit_bn_bwd', _row(0.0, 4000.0))
    assert r['bound'] == 'hbm' and r['unit'] == 'GB/s' and abs(r['frac'] - 0.5) < 1e-9


def test_conv_variants_priced_as_mfma():
    """the windowed / BatchNorm-fused conv entry points are MFMA work; pack / stem are not"""
    import bench
    for name in ('ewvit_conv2d_bwd_data_bn_win', 'ewvit_conv2d_fwd_bn_xf', 'ewvit_conv2d_bwd_weight_xf',
                 'ewvit_conv2d_fwd_bn', 'ewvit_conv2d_bwd_data_add', 'ewvit_gemm_tallk'):
        assert bench.roofline_for(name, _row(250.0, 0.0))['bound'] == 'mfma', name
    for name in ('ewvit_conv2d_pack_weights', 'ewvit_conv2d_stem_fwd'):
        assert bench.roofline_for(name, _row(0.0, 800.0))['bound'] == 'hbm', name


def test_pmc_patterns_cover_windowed_kernels():
    """every windowed conv kernel symbol maps to exactly one entry point (no double counting)"""
    import bench
    syms = ['void ewvit::conv_win_kernel<true, false, false, true, false>(ewvit::FwdArgs, long, long, int, int, int)',
            'void ewvit::conv_win_kernel<true, false, false, true, true>(ewvit::FwdArgs, long, long, int, int, int)',
            'void ewvit::conv_win_kernel<false, true, true, false, false>(ewvit::FwdArgs, long, long, int, int, int)',
            'void ewvit::conv_wgrad_win_kernel<true, true, true>(ewvit::WgradArgs, long, int, int, int, int)',
            'void ewvit::conv_wgrad_win_kernel<true, false, true>(ewvit::WgradArgs, long, int, int, int, int)',
            'void ewvit::conv_wgrad_1x1_kernel<2>(ewvit::WgradArgs, int, int)',
            'void ewvit::conv_win_kernel<false, true, false, false, false>(ewvit::FwdArgs, long, long, int, int, int)',
            'void ewvit::conv_win_kernel<true, false, false, false, false>(ewvit::FwdArgs, long, long, int, int, int)',
            'void ewvit::conv_win_kernel<false, false, false, false, false>(ewvit::FwdArgs, long, long, int, int, int)',
            'void ewvit::conv_glds_kernel<true, 128, 64, 3, 2, 4, false, true>(ewvit::FwdArgs, long, int, int, int)']
    for k in syms:
        owners = [e for e, pats in bench.ENTRY_KERNELS.items() if any(p in k for p in pats)]
        assert len(owners) == 1, (k, owners)
