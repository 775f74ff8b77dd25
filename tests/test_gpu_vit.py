"""The fused ViT encoder layer (csrc/vit.hip, ewvit.vit) against the module path of
network/sfe.py (the same reference semantics, sfe.py:72-85, on ewvit GEMM / LayerNorm /
attention kernels) and against the fp32 oracle.

The fused and module paths round the same operands to bf16 (LN outputs, q/k/v, the attention
output, h, dh, g1, dqkv) and draw the same to_out dropout mask (host seed + device counter,
index row * 512 + col); they differ in fp32 summation order only (split-K vs per-wave K
halves, column sums).  Bounds: outputs max |err| <= 2e-3 of scale and cosine >= 0.99999, every
parameter and the input gradient cosine >= 0.9999 with the norm within 0.3 %, with dropout on
and off, for 64 / 37 / 8 / 1 frames.  Against the oracle (fp32 CPU restatement): the bf16
bounds of the module path's own tests (2e-2 of scale, cosine >= 0.999 / gradients 0.99).
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _cos(a, b):
    a, b = a.detach().double().flatten(), b.detach().double().flatten()
    return float(a @ b / (a.norm() * b.norm() + 1e-30))


def _vit(drop, seed=0):
    from network.sfe import Transformer
    torch.manual_seed(seed)
    m = Transformer(512, 2, 8, 64, 2048, drop).to(DEV)
    with torch.no_grad():            # non-trivial LayerNorm affine / biases
        for n, p in m.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.1)
    return m


def _run(m, x0, fused, monkeypatch, seed=11):
    import ewvit
    monkeypatch.setenv('EWVIT_VIT_FUSED', '1' if fused else '0')
    calls = {}
    real = ewvit._lib.call

    def count(name, *a, **k):
        calls[name] = calls.get(name, 0) + 1
        return real(name, *a, **k)
    monkeypatch.setattr(ewvit._lib, 'call', count)
    x = x0.clone().requires_grad_(True)
    torch.manual_seed(seed)                  # the to_out dropout's host seeds
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = m(x)
    g = torch.Generator().manual_seed(5)
    w = torch.randn(y.shape, generator=g).to(DEV)
    (y.float() * w).sum().backward()
    torch.cuda.synchronize()
    monkeypatch.undo()
    grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    return y.detach().float(), x.grad.clone(), grads, calls


@pytest.mark.parametrize('N', [64, 37, 8, 1])
@pytest.mark.parametrize('drop', [0.0, 0.15])
def test_vit_layer_matches_module_path(N, drop, monkeypatch):
    m0 = _vit(drop).train()
    g = torch.Generator().manual_seed(N)
    x0 = (torch.randn(N, 2, 512, generator=g) * 1.5 + 0.3).to(DEV)
    a, b = copy.deepcopy(m0), copy.deepcopy(m0)
    ya, dxa, ga, ca = _run(a, x0, True, monkeypatch)
    yb, dxb, gb, cb = _run(b, x0, False, monkeypatch)
    assert ca.get('ewvit_vit_layer_fwd') == 2 and ca.get('ewvit_vit_layer_bwd') == 2, ca
    assert 'ewvit_vit_layer_fwd' not in cb and cb.get('ewvit_gemm', 0) > 0, cb
    scale = float(yb.abs().max())
    err = float((ya - yb).abs().max())
    assert err <= 2e-3 * scale and _cos(ya, yb) >= 0.99999, (err, scale, _cos(ya, yb))
    assert _cos(dxa, dxb) >= 0.9999
    assert abs(float(dxa.norm() / dxb.norm()) - 1) < 3e-3
    for n in gb:
        c = _cos(ga[n], gb[n])
        r = float(ga[n].norm() / gb[n].norm())
        assert c >= 0.9999 and abs(r - 1) < 3e-3, (n, c, r)


def test_vit_layer_eval_and_dropout_mask_per_replay(monkeypatch):
    """Eval mode: no dropout (two calls equal); training mode: the mask follows the device step
    counter (a new mask per advance), and the module path draws the same one."""
    import ewvit
    m = _vit(0.15).eval()
    x0 = torch.randn(16, 2, 512, device=DEV)
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
        y1, y2 = m(x0), m(x0)
    assert torch.equal(y1, y2)
    m.train()
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
        torch.manual_seed(3)
        a = m(x0)
        ewvit._lib.rng_advance(torch.device(DEV))
        torch.manual_seed(3)
        b = m(x0)
    assert not torch.equal(a, b)


def test_vit_layer_vs_oracle():
    """The fused path against the fp32 CPU restatement of sfe.Transformer (oracle/model.py)."""
    from oracle import model as om
    from oracle.weights import apply_recipe
    from network import sfe
    o = apply_recipe(om.Transformer(512, 2, 8, 64, 2048, 0.0), 3)
    p = sfe.Transformer(512, 2, 8, 64, 2048, 0.0)
    p.load_state_dict(o.state_dict())
    p = p.to(DEV)
    t = torch.randn(64, 2, 512, generator=torch.Generator().manual_seed(1))
    to, tp = t.clone().requires_grad_(True), t.to(DEV).requires_grad_(True)
    yo = o(to)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        yp = p(tp)
    w = torch.randn(yo.shape, generator=torch.Generator().manual_seed(2))
    (yo * w).sum().backward()
    (yp.float() * w.to(DEV)).sum().backward()
    scale = float(yo.abs().max())
    assert float((yp.detach().cpu() - yo.detach()).abs().max()) < 2e-2 * scale
    assert _cos(yp.cpu(), yo) >= 0.999
    assert _cos(tp.grad.cpu(), to.grad) >= 0.99
    for (n, a), (_, b) in zip(o.named_parameters(), p.named_parameters()):
        assert _cos(b.grad.cpu(), a.grad) >= 0.99, n


@pytest.mark.parametrize('B', [64, 13, 1])
def test_embed_matches_torch(B):
    """ewvit.vit.embed (CLS concat + pos_embedding[0:B] + emb dropout, sfe.py:155-160) against
    the torch expression; with dropout every element is 0 or the reference / (1 - p), and the
    backward applies the forward's mask."""
    import ewvit
    g = torch.Generator().manual_seed(B)
    y = torch.randn(B, 1, 512, generator=g).to(DEV)
    cls = torch.randn(1, 1, 512, generator=g).to(DEV)
    pos = torch.randn(64, 1, 512, generator=g).to(DEV)
    w = torch.randn(B, 2, 512, generator=g).to(DEV)
    ya, ca, pa = [t.clone().requires_grad_(True) for t in (y, cls, pos)]
    yb, cb, pb = [t.clone().requires_grad_(True) for t in (y, cls, pos)]
    ta = ewvit.vit.embed(ya, ca, pa, 0.0)
    tb = torch.cat((cb.expand(B, -1, -1), yb), 1) + pb[0:B]
    assert torch.equal(ta, tb)
    (ta * w).sum().backward()
    (tb * w).sum().backward()
    torch.testing.assert_close(ya.grad, yb.grad, rtol=0, atol=0)
    torch.testing.assert_close(pa.grad, pb.grad, rtol=0, atol=0)
    torch.testing.assert_close(ca.grad, cb.grad, rtol=1e-6, atol=1e-5)
    p = 0.15
    yd, cd, pd = [t.clone().requires_grad_(True) for t in (y, cls, pos)]
    td = ewvit.vit.embed(yd, cd, pd, p)
    keep = td != 0
    frac = float(keep.float().mean())
    assert abs(frac - (1 - p)) < 0.05 if B > 4 else True
    torch.testing.assert_close(td[keep], (tb.detach() / (1 - p))[keep], rtol=1e-6, atol=1e-6)
    (td * w).sum().backward()
    m = keep.float() / (1 - p)
    torch.testing.assert_close(yd.grad, (w * m)[:, 1:], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(pd.grad[0:B], (w * m).sum(1, keepdim=True), rtol=1e-6, atol=1e-6)
    assert float(pd.grad[B:].abs().max()) == 0.0 if B < 64 else True


@pytest.mark.parametrize('M', [64, 37, 1])
def test_tallk_gemm_patch_embedding_shape(M):
    """ewvit_gemm_tallk (patch_to_embedding's forward, sfe.py:155: [M, 62720] x [62720, 512] +
    bias) against torch fp32 on the same bf16-rounded operands (fp32 accumulation, different
    summation order: 1e-4 of scale) and against the generic split-K GEMM it replaces."""
    import ewvit
    g = torch.Generator().manual_seed(M)
    K, N = 62720, 512
    x = torch.randn(M, K, generator=g).to(DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.01).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    y = torch.empty(M, N, device=DEV)
    ewvit.mm_nt(x, w, y, bias=b)
    ref = x.float() @ w.to(torch.bfloat16).float().t() + b
    scale = float(ref.abs().max())
    assert float((y - ref).abs().max()) <= 1e-4 * scale
    y2 = torch.empty_like(y)
    ewvit.mm_nt(x, w, y2, bias=b, splitk=64)            # the generic split-K path
    assert float((y - y2).abs().max()) <= 1e-4 * scale


@pytest.mark.parametrize('N', [64, 37, 1])
def test_vit_layer_mxfp8_matches_module_path(N, monkeypatch):
    """fp8 token GEMMs (network.set_gemm_precision 'fp8', configs[4]): the fused layer on MXFP8
    operands (ewvit_vit_pack_mx + the MX kernels of csrc/vit.hip) against the module path, whose
    Linears run ewvit_gemm_mx8 — the same block format, quantized from the same activations
    except where the fused kernels keep them in fp32 (LayerNorm outputs, the attention output,
    the LN2-backward gradient) and the module path has them in bf16, so single e4m3 roundings
    differ.  Bounds: outputs 3e-2 of scale / cosine >= 0.999, gradients cosine >= 0.995 with
    norms within 2 %; no bf16 GEMM runs on either side."""
    from network import set_gemm_precision
    m0 = _vit(0.0).train()
    assert set_gemm_precision(m0, 'fp8') == 8
    g = torch.Generator().manual_seed(N + 1)
    x0 = (torch.randn(N, 2, 512, generator=g) * 1.5 + 0.3).to(DEV)
    a, b = copy.deepcopy(m0), copy.deepcopy(m0)
    ya, dxa, ga, ca = _run(a, x0, True, monkeypatch)
    yb, dxb, gb, cb = _run(b, x0, False, monkeypatch)
    assert ca.get('ewvit_vit_layer_fwd') == 2 and ca.get('ewvit_vit_pack_mx') == 1, ca
    assert 'ewvit_gemm' not in ca and 'ewvit_gemm' not in cb and cb.get('ewvit_gemm_mx8', 0) >= 24, (ca, cb)
    scale = float(yb.abs().max())
    err = float((ya - yb).abs().max())
    assert err <= 3e-2 * scale and _cos(ya, yb) >= 0.999, (err, scale, _cos(ya, yb))
    assert _cos(dxa, dxb) >= 0.995
    for n in gb:
        c = _cos(ga[n], gb[n])
        r = float(ga[n].norm() / gb[n].norm())
        assert c >= 0.995 and abs(r - 1) < 2e-2, (n, c, r)
