"""GPU parity of every ewvit kernel, called through the C-ABI (via ewvit.ops).

DWT / upsample are checked against the oracle (numpy restatement pinned to
pywt and the reference) and the pywt golden fixture; GEMM / LayerNorm /
attention against plain torch fp32 on the same bf16-rounded operands.
Tolerances are stated per test:
* DWT fp32 out: 1e-6 abs (identical op order, fp32);  bf16 out: one bf16 ulp.
* GEMM: fp32 accumulate of bf16 operands vs fp32 torch on the same bf16 values:
  rtol 2e-4 of the output scale (summation-order differences only).
* LayerNorm fp32: 2e-5;  attention (bf16 I/O): 1e-2 of scale.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail('no ROCm GPU visible')
    import ewvit
    ewvit.load_library()


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-12))


# ---------------------------------------------------------------- DWT
@pytest.mark.parametrize('shape,levels', [((64, 3, 224, 224), 3), ((2, 3, 64, 64), 2), ((1, 2, 13, 10), 2),
                                          ((3, 1, 33, 47), 3), ((1, 1, 2, 2), 1), ((2, 3, 384, 384), 3)])
def test_dwt_vs_oracle_fp32(shape, levels):
    import ewvit
    from oracle import dwt as odwt
    x = torch.randn(*shape, generator=torch.Generator().manual_seed(1))
    ll, yhs = ewvit.dwt_haar(x.to(DEV), levels, out_dtype=torch.float32)
    ll_o, yh_o = odwt.haar_multilevel(x.numpy(), levels)
    np.testing.assert_allclose(ll.cpu().numpy(), ll_o, atol=1e-6, rtol=0)
    for a, b in zip(yhs, yh_o):
        np.testing.assert_allclose(a.cpu().numpy(), b, atol=1e-6, rtol=0)


def test_dwt_vs_pywt_golden(golden):
    import ewvit
    z = golden('dwt_pywt.npz')
    for name, L in (('a', 3), ('b', 3), ('odd', 2)):
        x = torch.from_numpy(z[f'{name}.x']).to(DEV)
        ll, yhs = ewvit.dwt_haar(x, L, out_dtype=torch.float32)
        for lv in range(1, L + 1):
            np.testing.assert_allclose(yhs[lv - 1].cpu().numpy(), z[f'{name}.L{lv}.yh'], atol=2e-6)
        np.testing.assert_allclose(ll.cpu().numpy(), z[f'{name}.L{L}.ll'], atol=2e-6)


def test_dwt_bf16_in_and_out():
    import ewvit
    from oracle import dwt as odwt
    x = torch.randn(4, 3, 96, 64, generator=torch.Generator().manual_seed(2)).to(torch.bfloat16)
    ll, yhs = ewvit.dwt_haar(x.to(DEV), 3, out_dtype=torch.bfloat16)
    ll_o, yh_o = odwt.haar_multilevel(x.float().numpy(), 3)
    for a, b in zip(yhs + [ll], yh_o + [ll_o]):
        a = a.float().cpu().numpy()
        assert np.abs(a - b).max() <= 2 ** -7 * max(np.abs(b).max(), 1.0)


def test_dwt_layout_roundtrip_energy():
    """Orthonormal Haar: the 3 bands + LL of each level keep the input energy
    (a size-independent property checked at the full 64x3x224x224 size)."""
    import ewvit
    x = torch.randn(64, 3, 224, 224, device=DEV)
    ll, yhs = ewvit.dwt_haar(x, 3, out_dtype=torch.float32)
    e_in = x.double().pow(2).sum()
    e_out = ll.double().pow(2).sum() + sum(y.double().pow(2).sum() for y in yhs)
    assert abs(float(e_out / e_in) - 1.0) < 1e-5


@pytest.mark.parametrize('shape,levels,out_hw', [((8, 3, 224, 224), 3, (112, 112)), ((2, 3, 64, 64), 2, (32, 32)),
                                                 ((2, 3, 64, 64), 1, (32, 32)), ((1, 2, 40, 24), 3, (20, 12))])
def test_hf_upsample_vs_oracle(shape, levels, out_hw):
    import ewvit
    from oracle import dwt as odwt
    x = torch.randn(*shape, generator=torch.Generator().manual_seed(3))
    up, _ = ewvit.dwt_hf_upsample(x.to(DEV), levels, out_hw, out_dtype=torch.float32, band_dtype=torch.float32)
    ref = odwt.hf_upsampled(x.numpy(), levels)            # [L, N, 3C, OH, OW]
    got = up.permute(0, 1, 4, 2, 3).cpu().numpy()          # [L, N, OH, OW, 3C] -> [L, N, 3C, OH, OW]
    np.testing.assert_allclose(got, ref, atol=2e-6, rtol=0)


def test_hf_upsample_bf16_is_rounded_fp32():
    import ewvit
    x = torch.randn(4, 3, 224, 224, device=DEV)
    a, _ = ewvit.dwt_hf_upsample(x, 3, (112, 112), out_dtype=torch.float32, band_dtype=torch.float32)
    b, _ = ewvit.dwt_hf_upsample(x, 3, (112, 112), out_dtype=torch.bfloat16, band_dtype=torch.bfloat16)
    assert rel_err(b.float(), a) < 2 ** -7


@pytest.mark.parametrize('shape,levels,odt,oc,xdt', [
    ((64, 3, 224, 224), 3, torch.bfloat16, 16, torch.float32),     # config 2's MWT front end
    ((6, 3, 96, 224), 3, torch.bfloat16, 16, torch.float32),
    ((4, 3, 224, 224), 3, torch.bfloat16, 16, torch.bfloat16),
    ((4, 3, 64, 64), 2, torch.float32, 9, torch.float32),
    ((2, 3, 40, 72), 3, torch.bfloat16, 16, torch.float32),        # 20 level-1 rows: a ragged strip
    ((2, 3, 32, 48), 1, torch.float32, 9, torch.float32),
    ((3, 3, 8, 200), 3, torch.float32, 12, torch.float32)])
def test_dwt_hf_fused_equals_two_launch_path(shape, levels, odt, oc, xdt):
    """ewvit_dwt_hf_upsample_fused (one launch, bands on chip) gives exactly the values of
    dwt_haar_fwd (bands rounded to the output type) + hf_upsample."""
    import ewvit
    from ewvit import _lib as L
    N, C, H, W = shape
    assert L.load().ewvit_dwt_hf_fused_ok(N, C, H, W, levels, H // 2, W // 2, oc)
    x = torch.randn(*shape, generator=torch.Generator().manual_seed(11)).to(DEV, xdt)
    got = torch.ops.ewvit.dwt_hf_fused(x, levels, odt, oc)
    ref, _ = ewvit.dwt_hf_upsample(x, levels, (H // 2, W // 2), out_dtype=odt, band_dtype=odt, out_channels=oc)
    assert got.shape == ref.shape == (levels, N, H // 2, W // 2, oc)
    assert torch.equal(got, ref)


def test_dwt_hf_fused_vs_oracle_and_dispatch():
    """The fused path against the oracle (fp32), and dwt_hf_features' dispatch: shapes the
    fused kernel does not take (odd sizes, 4 levels, C != 3) run the two launches."""
    import ewvit
    from ewvit import _lib as L
    from oracle import dwt as odwt
    x = torch.randn(8, 3, 224, 224, generator=torch.Generator().manual_seed(3))
    up = ewvit.dwt_hf_features(x.to(DEV), 3, (112, 112), out_dtype=torch.float32)
    ref = odwt.hf_upsampled(x.numpy(), 3)
    np.testing.assert_allclose(up.permute(0, 1, 4, 2, 3).cpu().numpy(), ref, atol=2e-6, rtol=0)
    lib = L.load()
    for shape, lv, oc in [((2, 3, 42, 40), 3, 16), ((2, 3, 64, 64), 4, 16), ((2, 2, 64, 64), 2, 6),
                          ((1, 3, 16, 416), 3, 16), ((2, 3, 384, 384), 3, 16)]:
        N, C, H, W = shape
        assert not lib.ewvit_dwt_hf_fused_ok(N, C, H, W, lv, H // 2, W // 2, oc)
        xs = torch.randn(*shape, device=DEV)
        a = ewvit.dwt_hf_features(xs, lv, (H // 2, W // 2), out_dtype=torch.bfloat16, out_channels=oc)
        b, _ = ewvit.dwt_hf_upsample(xs, lv, (H // 2, W // 2), out_dtype=torch.bfloat16, band_dtype=torch.bfloat16,
                                     out_channels=oc)
        assert torch.equal(a, b)


# ---------------------------------------------------------------- GEMM
def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize('M,N,K', [(128, 1536, 512), (64, 512, 62720), (77, 93, 45), (1, 3, 64), (130, 2048, 512),
                                   (512, 1000, 64)])
@pytest.mark.parametrize('adt', [torch.float32, torch.bfloat16])
def test_gemm_nt_nn_tn(M, N, K, adt):
    import ewvit
    g = torch.Generator().manual_seed(M * 7 + N)
    X = torch.randn(M, K, generator=g).to(adt)
    W = torch.randn(N, K, generator=g)
    Xd, Wd = X.to(DEV), W.to(DEV)
    ref = _bf(X.float()) @ _bf(W).T
    y = ewvit.mm_nt(Xd, Wd, torch.empty(M, N, device=DEV))
    assert rel_err(y, ref) < 2e-4
    G = torch.randn(M, N, generator=g)
    dx = ewvit.mm_nn(G.to(DEV), Wd, torch.empty(M, K, device=DEV))
    assert rel_err(dx, _bf(G) @ _bf(W)) < 2e-4
    dw = ewvit.mm_tn(G.to(DEV), Xd, torch.empty(N, K, device=DEV))
    assert rel_err(dw, _bf(G).T @ _bf(X.float())) < 2e-4


@pytest.mark.parametrize('splitk', [1, 3, 16])
def test_gemm_splitk_and_epilogues(splitk):
    import ewvit
    g = torch.Generator().manual_seed(11)
    M, N, K = 70, 200, 3000
    X, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    pre = _bf(X) @ _bf(W).T + b
    # GELU + aux, residual
    y = torch.empty(M, N, device=DEV)
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ewvit.mm_nt(X.to(DEV), W.to(DEV), y, bias=b.to(DEV), act=1, aux=aux, resid=R.to(DEV), ldr=N, splitk=splitk)
    assert rel_err(y, torch.nn.functional.gelu(pre) + R) < 5e-4
    assert rel_err(aux.float(), pre) < 2 ** -7
    # ReLU, bf16 output
    yb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ewvit.mm_nt(X.to(DEV), W.to(DEV), yb, bias=b.to(DEV), act=2, splitk=splitk)
    assert rel_err(yb.float(), torch.relu(pre)) < 2 ** -7
    # act 3: multiply by GELU'(aux)
    y3 = torch.empty(M, N, device=DEV)
    ewvit.mm_nt(X.to(DEV), W.to(DEV), y3, act=3, aux=aux, splitk=splitk)
    h = aux.float().cpu().requires_grad_(True)
    torch.nn.functional.gelu(h).sum().backward()
    assert rel_err(y3, (_bf(X) @ _bf(W).T) * h.grad) < 5e-4
    # beta accumulation into f32 C
    c0 = torch.randn(M, N, generator=g)
    yc = c0.clone().to(DEV)
    ewvit.mm_nt(X.to(DEV), W.to(DEV), yc, beta=1.0, splitk=splitk)
    assert rel_err(yc, c0 + _bf(X) @ _bf(W).T) < 5e-4


def test_gemm_dropout_mask_statistics_and_backward_consistency():
    import ewvit
    from ewvit import _lib as L
    M, N, K = 256, 512, 64
    X = torch.randn(M, K, device=DEV)
    W = torch.randn(N, K, device=DEV)
    y0 = ewvit.mm_nt(X, W, torch.empty(M, N, device=DEV))
    y = ewvit.mm_nt(X, W, torch.empty(M, N, device=DEV), drop_p=0.15, seed=1234)
    kept = (y != 0)
    frac = kept.float().mean().item()
    assert abs(frac - 0.85) < 0.01
    torch.testing.assert_close(y[kept], (y0 / 0.85)[kept], rtol=1e-5, atol=1e-5)
    # backward regenerates the same mask from the seed
    g = torch.ones(M, N, device=DEV)
    L.call('ewvit_dropout_bwd', L.ptr(g), 0, M, N, N, 0.15, 1234, None, L.stream(g))
    assert torch.equal(g != 0, kept)
    # with a device step counter: same mask while the counter holds, a new one after it moves
    off = torch.full((1,), 5, dtype=torch.int64, device=DEV)
    y5 = ewvit.mm_nt(X, W, torch.empty(M, N, device=DEV), drop_p=0.15, seed=1234, seed_offset=off)
    g = torch.ones(M, N, device=DEV)
    L.call('ewvit_dropout_bwd', L.ptr(g), 0, M, N, N, 0.15, 1234, L.ptr(off), L.stream(g))
    assert torch.equal(g != 0, y5 != 0) and not torch.equal(y5 != 0, kept)


def test_colsum():
    import ewvit
    X = torch.randn(1000, 300, device=DEV)
    out = torch.empty(300, device=DEV)
    ewvit.colsum(X, out)
    assert rel_err(out, X.sum(0)) < 1e-5


# ---------------------------------------------------------------- LayerNorm / attention
@pytest.mark.parametrize('M,D', [(128, 512), (64, 128), (5, 1000)])
def test_layernorm_fwd_bwd(M, D):
    import ewvit
    x = torch.randn(M, D, dtype=torch.float64) * 3 + 1
    gm, bt = torch.randn(D, dtype=torch.float64), torch.randn(D, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    gr, br = gm.clone().requires_grad_(True), bt.clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-5)
    dy = torch.randn(M, D, dtype=torch.float64)
    yr.backward(dy)
    xd = x.float().to(DEV).requires_grad_(True)
    gd, bd = gm.float().to(DEV).requires_grad_(True), bt.float().to(DEV).requires_grad_(True)
    y = ewvit.layer_norm(xd, gd, bd, 1e-5, out_dtype=torch.float32)
    y.backward(dy.float().to(DEV))
    assert rel_err(y, yr) < 2e-5
    assert rel_err(xd.grad, xr.grad) < 2e-5
    assert rel_err(gd.grad, gr.grad) < 2e-5
    assert rel_err(bd.grad, br.grad) < 2e-5


def _ref_attn(q, k, v, H, d, scale):
    B, nq, _ = q.shape
    nk = k.shape[1]
    qh = q.view(B, nq, H, d).transpose(1, 2)
    kh = k.view(B, nk, H, d).transpose(1, 2)
    vh = v.view(B, nk, H, d).transpose(1, 2)
    p = torch.softmax(qh @ kh.transpose(-1, -2) * scale, -1)
    return (p @ vh).transpose(1, 2).reshape(B, nq, H * d)


@pytest.mark.parametrize('packed,B,n,nk,H,d', [(True, 64, 2, 2, 8, 64), (False, 64, 1, 2, 4, 32), (True, 3, 5, 5, 2, 128),
                                               (False, 7, 3, 8, 3, 16)])
def test_attention_fwd_bwd(packed, B, n, nk, H, d):
    import ewvit
    g = torch.Generator().manual_seed(5)
    inner = H * d
    scale = d ** -0.5
    if packed:
        qkv = torch.randn(B, n, 3 * inner, generator=g).to(torch.bfloat16)
        q, k, v = qkv.float().split(inner, -1)
    else:
        qt = torch.randn(B, n, inner, generator=g).to(torch.bfloat16)
        kv = torch.randn(B, nk, 2 * inner, generator=g).to(torch.bfloat16)
        q = qt.float()
        k, v = kv.float().split(inner, -1)
    q, k, v = (t.clone().requires_grad_(True) for t in (q, k, v))
    ref = _ref_attn(q, k, v, H, d, scale)
    do = torch.randn(ref.shape, generator=g).to(torch.bfloat16)
    ref.backward(do.float())
    if packed:
        src = qkv.to(DEV).requires_grad_(True)
        o = ewvit.attention_packed(src, H, d, scale)
        o.backward(do.to(DEV))
        dq, dk, dv = src.grad.float().cpu().split(inner, -1)
    else:
        qs, kvs = qt.to(DEV).requires_grad_(True), kv.to(DEV).requires_grad_(True)
        o = ewvit.attention_cross(qs, kvs, H, d, scale)
        o.backward(do.to(DEV))
        dq = qs.grad.float().cpu()
        dk, dv = kvs.grad.float().cpu().split(inner, -1)
    assert rel_err(o.float(), ref) < 1e-2
    assert rel_err(dq, q.grad) < 1.5e-2
    assert rel_err(dk, k.grad) < 1.5e-2
    assert rel_err(dv, v.grad) < 1.5e-2


def test_linear_autograd_matches_torch():
    import ewvit
    g = torch.Generator().manual_seed(9)
    x = torch.randn(4, 2, 512, generator=g)
    W = torch.randn(2048, 512, generator=g) / 512 ** 0.5
    b = torch.randn(2048, generator=g)
    r = torch.randn(4, 2, 2048, generator=g)
    xr, Wr, br, rr = (t.clone().requires_grad_(True) for t in (x, W, b, r))
    yr = torch.nn.functional.gelu(_bf(xr) @ _bf(Wr).T + br) + rr
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xd, Wd, bd, rd = (t.to(DEV).requires_grad_(True) for t in (x, W, b, r))
    y = ewvit.linear(xd, Wd, bd, act=1, resid=rd)
    y.backward(dy.to(DEV))
    assert rel_err(y, yr) < 1e-3
    # gradients see bf16-rounded operands inside the GEMMs: 1e-2 of scale
    for a, b_ in ((xd, xr), (Wd, Wr), (bd, br), (rd, rr)):
        assert rel_err(a.grad, b_.grad) < 1e-2


def test_bad_arguments_raise_on_gpu():
    import ewvit
    with pytest.raises(RuntimeError, match='levels'):
        ewvit.dwt_haar(torch.randn(1, 1, 8, 8, device=DEV), 6)
    with pytest.raises(TypeError):
        ewvit.attention_packed(torch.randn(2, 2, 12, device=DEV), 2, 2, 1.0)


# ---------------------------------------------------------------- depthwise conv
@pytest.mark.parametrize('N,C,H,stride', [(64, 960, 14, 1), (4, 256, 28, 2), (3, 1536, 7, 1), (2, 64, 15, 2),
                                          (1, 8, 5, 1), (8, 960, 14, 2), (2, 48, 9, 2), (3, 16, 3, 2)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_depthwise_fwd_bwd_vs_torch(N, C, H, stride, dtype):
    """vs torch fp32 conv2d(groups=C) on the same (rounded) values."""
    import ewvit
    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(N, C, H, H, generator=g).to(dtype)
    w = torch.randn(C, 1, 3, 3, generator=g)
    dy_shape = (N, C, (H - 1) // stride + 1, (H - 1) // stride + 1)
    dy = torch.randn(dy_shape, generator=g).to(dtype)
    xr, wr = x.float().clone().requires_grad_(True), w.clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, stride=stride, padding=1, groups=C)
    yr.backward(dy.float())
    xd = x.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = ewvit.dwconv3x3(xd, wd, stride, 1)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == dtype
    y.backward(dy.to(DEV))
    tol = 1e-5 if dtype == torch.float32 else 2 ** -7
    assert rel_err(y.float(), yr) < tol
    assert rel_err(xd.grad.float(), xr.grad) < tol
    assert rel_err(wd.grad, wr.grad) < 1e-5 if dtype == torch.float32 else rel_err(wd.grad, wr.grad) < 1e-4



def test_hf_upsample_padded_channels():
    """out_channels > 3C: the bands in channels 0..3C-1 (the unpadded result up to one
    bf16 rounding: the vectorised store path may contract the lerp differently),
    exact zeros after — the 16-channel input of the MWT seperate conv."""
    import ewvit
    x = torch.randn(3, 3, 40, 36, generator=torch.Generator().manual_seed(5)).to(DEV)
    a, _ = ewvit.dwt_hf_upsample(x, 3, (20, 18), out_dtype=torch.bfloat16, band_dtype=torch.bfloat16)
    b, _ = ewvit.dwt_hf_upsample(x, 3, (20, 18), out_dtype=torch.bfloat16, band_dtype=torch.bfloat16,
                                 out_channels=16)
    assert b.shape[-1] == 16
    d = (b[..., :9].float() - a.float()).abs()
    assert float((d / a.float().abs().clamp_min(1e-3)).max()) <= 2 ** -7
    assert float(b[..., 9:].abs().max()) == 0.0


@pytest.mark.parametrize('shape,dtype', [((4, 128, 56, 56), torch.bfloat16), ((3, 16, 9, 11), torch.float32),
                                         ((2, 64, 8, 8), torch.bfloat16)])
def test_maxpool2_matches_torch(shape, dtype):
    """ewvit.maxpool2 (csrc/pool.hip) vs nn.MaxPool2d(2): outputs bitwise, and the
    gradient routed to the same window element (ties included: integer-valued inputs
    make many; torch keeps the first maximum), odd sizes in floor mode."""
    import ewvit
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randint(-3, 4, shape, generator=g).to(dtype)           # many ties
    x[0, 0, 0, 0] = float('nan')
    xd = x.to(DEV).to(memory_format=torch.channels_last).requires_grad_(True)
    xr = x.clone().to(DEV).requires_grad_(True)
    y = ewvit.maxpool2(xd)
    yr = torch.nn.functional.max_pool2d(xr, 2)
    assert y.shape == yr.shape
    assert torch.equal(torch.nan_to_num(y.float(), 99.0), torch.nan_to_num(yr.float(), 99.0))
    dy = torch.randn(y.shape, generator=g).to(dtype).to(DEV)
    y.backward(dy)
    yr.backward(dy)
    assert torch.equal(xd.grad.float(), xr.grad.float())
