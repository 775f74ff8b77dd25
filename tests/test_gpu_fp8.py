"""fp8 e4m3 GEMMs (BASELINE.json configs[4]: "fp8 (e4m3) MFMA for attention/MLP GEMMs, bf16
DWT, 224x224 bs=128").

The fp8 format is MXFP8 (OCP MX): every run of 32 consecutive K elements of a row of A (a
column of B) shares one power-of-two E8M0 scale 2^X, X the smallest with max|run| <= 448 * 2^X,
and its elements are rounded to OCP e4m3fn (csrc/mx8.h; v_mfma_scale_f32_16x16x128_f8f6f4).

Kernel level (ewvit_gemm_mx8 through the C-ABI):
* the lane maps of the scaled MFMA in all three operand layouts, with exact integer data (every
  value and every block-scaled value exact in e4m3, every sum exact in fp32) — bit-exact;
* random operands against an emulation built on torch's own float8_e4m3fn cast (CPU, float64
  scales): only the accumulation differs (bound 1e-4 of scale), which also pins the rounding
  (RNE) of the hardware conversion to OCP e4m3fn and the block / scale placement: one block
  scaled 2x wrong moves the result by >= 1e-3 of scale at these K;
* split-K at the patch_to_embedding shape (M=64, N=512, K=62720).

Module level: the DAMA train step with network.set_gemm_precision(model, 'fp8') against the
fp32 oracle, bounded by an fp8 YARDSTICK measured in the test (the reference's own module
sequence on the GPU under torch's bf16 autocast with its 20 attention / MLP GEMMs' operands cast through
torch.float8_e4m3fn, per-tensor scaled, fp32 accumulation — forward and both backward GEMMs);
and the config-5 chunking (16 videos x 8 frames, batch_size=4 -> two 64-frame chunks) equal to
composing _process_frame per chunk.
"""
import copy

import pytest
import torch

from test_gpu_modules import cos, log

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _mx_q(X):
    """MXFP8 of X [R, K] along K (blocks of 32, zero-padded) in float64."""
    R, K = X.shape
    Kp = (K + 31) // 32 * 32
    x = torch.zeros(R, Kp, dtype=torch.float64)
    x[:, :K] = X.double()
    xb = x.view(R, Kp // 32, 32)
    amax = xb.abs().amax(-1).float()
    m, e = torch.frexp(amax)                      # amax = m 2^e, m in [0.5, 1)
    ea = e - 1
    X_ = torch.where(amax > 0, ea - 8 + (2 * m > 1.75).int(), torch.zeros_like(ea))
    s = torch.pow(2.0, X_.double()).unsqueeze(-1)
    q = (xb / s).float().to(torch.float8_e4m3fn).double() * s
    return q.view(R, Kp)[:, :K]


def _emulate(A, B):
    """A [M,K], B [K,N] fp32 CPU -> the MXFP8 product in float64."""
    return _mx_q(A) @ _mx_q(B.t()).t()


@pytest.mark.parametrize('layout', ['nt', 'nn', 'tn'])
def test_fp8_gemm_lane_maps_exact_integers(layout):
    import ewvit
    g = torch.Generator().manual_seed(1)
    M, N, K = 96, 80, 160
    A = torch.randint(-8, 9, (M, K), generator=g).float()
    B = torch.randint(-8, 9, (K, N), generator=g).float()
    A[3, 7] = 448.0                       # amax 448 -> scale 1: all values exact in e4m3
    B[5, 2] = -448.0
    ref = A.double() @ B.double()
    Ad, Bd = A.to(DEV), B.to(DEV)
    out = torch.empty(M, N, device=DEV)
    if layout == 'nt':       # B given as W[N, K] (nn.Linear forward)
        ewvit.mm_nt(Ad, Bd.t().contiguous(), out, fp8=True)
    elif layout == 'nn':     # dX = G[M, N'] @ W[N', K']
        ewvit.mm_nn(Ad, Bd.contiguous(), out, fp8=True)
    else:                    # dW = G^T X: A given m-contiguous
        ewvit.mm_tn(Ad.t().contiguous(), Bd.contiguous(), out, fp8=True)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu().double(), ref)


@pytest.mark.parametrize('M,N,K,spread', [(128, 1536, 512, 0), (64, 512, 2048, 0), (37, 100, 70, 0),
                                           (128, 512, 512, 6)])
def test_fp8_gemm_vs_torch_e4m3_emulation(M, N, K, spread):
    """spread 6: every 32-element block of A and W scaled by its own 10^U(-3, 3) — the block
    scales must follow the blocks (a per-tensor scale would flush the small blocks to zero)."""
    import ewvit
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g) * 3
    W = torch.randn(N, K, generator=g) * 0.05
    if spread:
        A = A * torch.pow(10.0, (torch.rand(M, K // 32, 1, generator=g) - 0.5) * spread).expand(M, K // 32, 32).reshape(M, K)
        W = W * torch.pow(10.0, (torch.rand(N, K // 32, 1, generator=g) - 0.5) * spread).expand(N, K // 32, 32).reshape(N, K)
    ref = _emulate(A, W.t())
    out = torch.empty(M, N, device=DEV)
    ewvit.mm_nt(A.to(DEV), W.to(DEV), out, fp8=True)
    # per output row, relative to that row's scale (rows differ by up to 10^6 under the spread)
    err = float(((out.cpu().double() - ref).abs().amax(1) / ref.abs().amax(1)).max())
    log('fp8_vs_emulation', err, 1e-4)
    assert err <= 1e-4, err
    # and the e4m3 product is an approximation of the exact one (sanity of the scaling)
    exact = A.double() @ W.t().double()
    assert cos(out.cpu(), exact) > 0.995


def test_fp8_gemm_splitk_patch_embedding_shape():
    import ewvit
    g = torch.Generator().manual_seed(5)
    M, N, K = 64, 512, 62720
    X = torch.randn(M, K, generator=g).relu()          # backbone map after SiLU/ReLU-like
    W = torch.randn(N, K, generator=g) / K ** 0.5
    out = torch.empty(M, N, device=DEV)
    ewvit.mm_nt(X.to(DEV).bfloat16(), W.to(DEV), out, fp8=True)   # bf16 activations, fp32 master weight
    ref = _emulate(X.bfloat16().float(), W.t())
    err = float((out.cpu().double() - ref).abs().max()) / float(ref.abs().max())
    log('fp8_splitk_vs_emulation', err, 1e-4)
    assert err <= 1e-4, err


# The fp8 yardstick: what an fp8 run of the REFERENCE gives on this input —
# the oracle's module sequence on the GPU under torch's bf16 autocast (as the bf16 headline test
# measures its envelope), with the operands of the same 22 token GEMMs cast through
# torch.float8_e4m3fn with a per-tensor scale 448 / amax (the conventional fp8 recipe) and fp32
# accumulation, in the forward and in both backward GEMMs (dX = q(dY) q(W), dW = q(dY)^T q(X)).
# Runs on x and on 3 copies of x with 2^-8 relative input noise; the product passes a metric when
# its distance to the fp32 oracle is at most YARD_X x the furthest yardstick run's (max error of
# scale, and the cosine gap 1 - cos), inside fixed floors.
YARD_X = 1.5
FP8_FLOOR_ERR, FP8_FLOOR_COS, FP8_FLOOR_GCOS = 0.2, 0.99, 0.9


def _q8(t):
    """per-tensor e4m3 fake-quantisation (float32 result, values exactly the e4m3 grid x 1/s)"""
    t = t.float()
    amax = float(t.abs().max())
    s = 448.0 / amax if amax > 0 else 1.0
    return (t * s).clamp(-448, 448).to(torch.float8_e4m3fn).float() / s


class _Fp8Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        xq, wq = _q8(x), _q8(w)
        ctx.save_for_backward(xq, wq)
        ctx.has_b = b is not None
        y = xq @ wq.t()
        if b is not None:
            y = y + b.float()
        return y.to(torch.bfloat16) if torch.is_autocast_enabled() else y

    @staticmethod
    def backward(ctx, g):
        xq, wq = ctx.saved_tensors
        g2 = g.float().reshape(-1, g.shape[-1])
        gq = _q8(g2)
        dx = (gq @ wq).reshape(*g.shape[:-1], wq.shape[1])
        dw = gq.t() @ xq.reshape(-1, xq.shape[-1])
        db = g2.sum(0) if ctx.has_b else None
        return dx, dw, db


def _fp8_yardstick(o, names, x, batch_size):
    """The oracle o (CPU fp32) copied to the GPU, the Linears `names` on _Fp8Linear, run under
    bf16 autocast: outputs and parameter gradients (fp32 on the CPU)."""
    import types
    g = copy.deepcopy(o).to(DEV).train()
    mods = dict(g.named_modules())
    for n in names:
        m = mods[n]
        m.forward = types.MethodType(lambda self, t: _Fp8Linear.apply(t, self.weight, self.bias), m)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        r = g(x.to(DEV), batch_size=batch_size)
    w = {k: torch.randn(v.shape, generator=torch.Generator().manual_seed(i)) for i, (k, v) in enumerate(sorted(r.items()))}
    sum((r[k].float() * w[k].to(DEV)).sum() for k in r).backward()
    torch.cuda.synchronize()
    return ({k: v.detach().float().cpu() for k, v in r.items()},
            {n: p.grad.detach().cpu() for n, p in g.named_parameters() if p.grad is not None})


def _errs(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).abs().max()) / max(float(b.abs().max()), 1e-6), cos(a, b)


def test_dama_train_step_fp8_vs_oracle_and_fp8_yardstick():
    """DAMA train step (2 videos x 8 frames, batch_size 4: two 8-frame chunks) with the 20
    attention / MLP GEMMs on MXFP8 (the fused ViT layer and head kernels) against the fp32
    oracle, bounded by the in-test fp8 yardstick (the same 20 Linears per-tensor e4m3)."""
    from network import dama, set_gemm_precision
    from oracle import model as om
    from oracle.weights import recipe_input
    from test_gpu_modules import pair
    torch.manual_seed(0)
    p, o = pair(dama.DAMA, om.DAMA, (3, 128, 4, 3, 8), 14)
    assert set_gemm_precision(p, 'fp8') == 20
    names = [n for n, m in p.named_modules() if getattr(m, 'gemm_precision', 'bf16') == 'fp8']
    assert len(names) == 20
    p.train(); o.train()
    x = recipe_input((2, 8, 3, 224, 224), seed=4242)
    yards = [_fp8_yardstick(o, names, x, 4)]
    for sd_ in (5, 6, 7):
        gj = torch.Generator().manual_seed(sd_)
        yards.append(_fp8_yardstick(o, names, x * (1 + (torch.rand(x.shape, generator=gj) * 2 - 1) * 2.0 ** -8), 4))
    ro = o(x, batch_size=4)
    import ewvit
    calls = {}
    real = ewvit._lib.call

    def count(name, *a, **k):
        calls[name] = calls.get(name, 0) + 1
        return real(name, *a, **k)
    ewvit._lib.call = count
    try:
        with torch.autocast('cuda', dtype=torch.bfloat16):
            rp = p(x.to(DEV), batch_size=4)
        w = {k: torch.randn(v.shape, generator=torch.Generator().manual_seed(i)) for i, (k, v) in enumerate(sorted(ro.items()))}
        sum((ro[k] * w[k]).sum() for k in ro).backward()
        sum((rp[k].float() * w[k].to(DEV)).sum() for k in rp).backward()
        torch.cuda.synchronize()
    finally:
        ewvit._lib.call = real
    # the fused MX token kernels ran; the generic GEMMs left are the bf16 patch_to_embedding /
    # feat_map ones (dgrad + wgrad of patch_to_embedding, forward + dgrad + wgrad of feat_map per
    # chunk; the patch_to_embedding forward is ewvit_gemm_tallk) and the FeedForward's second
    # MXFP8 GEMM per layer and chunk in the forward
    print(calls)
    assert calls.get('ewvit_vit_pack_mx') == 2 and calls.get('ewvit_head_fwd') == 2, calls
    assert calls.get('ewvit_gemm', 0) <= 10 and calls.get('ewvit_gemm_mx8', 0) <= 12, calls
    fails = []

    def judge(kind, prod, ys, floor_err, floor_cos):
        ye = max(y[0] for y in ys)
        yc = min(y[1] for y in ys)
        ok = prod[0] <= max(YARD_X * ye, 1e-3) and (1 - prod[1]) <= max(YARD_X * (1 - yc), 1e-5) \
            and prod[0] <= floor_err and prod[1] >= floor_cos
        print(f'{"" if ok else "FAIL "}{kind:55s} product err {prod[0]:.4f} cos {prod[1]:.6f} | fp8 yardstick: '
              f'max err {ye:.4f} min cos {yc:.6f}')
        log('fp8_err_of_scale:' + kind, prod[0], YARD_X * ye)
        log('fp8_cos:' + kind, prod[1], 1 - YARD_X * (1 - yc))
        if not ok:
            fails.append((kind, prod, ye, yc))
    for k in ro:
        judge(k, _errs(rp[k], ro[k]), [_errs(y[0][k], ro[k]) for y in yards], FP8_FLOOR_ERR, FP8_FLOOR_COS)
    pp, oo = dict(p.named_parameters()), dict(o.named_parameters())
    for n in ('sfe.patch_to_embedding.weight', 'sfe.transformer.layers.0.0.fn.to_qkv.weight',
              'sfe.transformer.layers.1.1.fn.net.0.weight', 'sfe.transformer.layers.1.1.fn.net.3.weight',
              'cross_att.layers.1.3.to_kv.weight', 'cross_att.layers.0.1.to_out.0.weight', 'sfe.feat_map.0.weight',
              'mwt.multiscale_fusion.0.weight', 'sfe.efficient_net.features.7.0.weight'):
        pc = (0.0, cos(pp[n].grad, oo[n].grad))
        judge('grad ' + n, pc, [(0.0, cos(y[1][n], oo[n].grad)) for y in yards], 1.0, FP8_FLOOR_GCOS)
    assert not fails, fails


def test_set_gemm_precision_targets():
    from network import set_gemm_precision
    from network.model import DeepfakeDetector
    m = DeepfakeDetector(3, 128, 4)
    assert set_gemm_precision(m, 'fp8') == 20
    assert m.dama.sfe.transformer.layers[0][0].fn.to_qkv.gemm_precision == 'fp8'
    assert getattr(m.dama.sfe.patch_to_embedding, 'gemm_precision', 'bf16') == 'bf16'
    assert getattr(m.dama.sfe.feat_map[0], 'gemm_precision', 'bf16') == 'bf16'
    assert getattr(m.classifier[0], 'gemm_precision', 'bf16') == 'bf16'
    assert getattr(m.dama.gate_net[2], 'gemm_precision', 'bf16') == 'bf16'
    with pytest.raises(ValueError):
        set_gemm_precision(m, 'fp4')


def test_config5_two_chunks_equal_per_chunk_composition():
    """x [16, 8, 3, 224, 224], batch_size=4 (dama.py:179-199): two 64-frame chunks, per-video
    sums over chunks / K — equal to composing _process_frame on each chunk by hand."""
    from network import dama, set_gemm_precision
    torch.manual_seed(0)
    m = dama.DAMA(3, 128, 4, 3, 4).to(DEV).to(memory_format=torch.channels_last).eval()
    set_gemm_precision(m, 'fp8')
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(16, 8, 3, 224, 224, device=DEV, generator=g)
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
        out = m(x, batch_size=4)
        acc = None
        for s in (0, 4):
            f = m._process_frame(x[:, s:s + 4].flatten(0, 1))
            part = {k: v.float().view(16, -1, 128).sum(1) for k, v in f.items()}
            acc = part if acc is None else {k: acc[k] + part[k] for k in acc}
    for k in out:
        assert out[k].shape == (16, 128)
        torch.testing.assert_close(out[k].float(), acc[k] / 8, rtol=1e-5, atol=1e-6)
