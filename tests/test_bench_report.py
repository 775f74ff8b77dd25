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
