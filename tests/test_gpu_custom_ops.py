"""torch.ops.ewvit.* on the GPU (SURVEY §8b "registered via torch.library"):
torch.library.opcheck on every hot-path op (schema, fake-tensor agreement with the real
kernel, autograd registration, AOT dispatch), and torch.compile(fullgraph=True) of the ViT
block and the cross-attention layer, forward + backward, equal to eager."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _rand(*shape, dtype=torch.float32, rg=False):
    return torch.randn(*shape, device=DEV, dtype=dtype).requires_grad_(rg)


def _cases():
    x = _rand(16, 2, 64, rg=True)
    w = _rand(96, 64, rg=True)
    b = _rand(96, rg=True)
    qkv = _rand(8, 2, 3 * 4 * 16, dtype=torch.bfloat16, rg=True)
    q = _rand(8, 1, 4 * 16, dtype=torch.bfloat16, rg=True)
    kv = _rand(8, 2, 2 * 4 * 16, dtype=torch.bfloat16, rg=True)
    frames = _rand(2, 3, 32, 32)
    ll, yh = torch.ops.ewvit.dwt_haar(frames, 2, torch.bfloat16)
    return {
        'linear': (torch.ops.ewvit.linear.default, (x, w, b, 0, 0.0, 0, None, torch.float32, False, False)),
        'linear_gelu': (torch.ops.ewvit.linear.default, (x, w, b, 1, 0.0, 0, None, torch.bfloat16, False, True)),
        'linear_fp8': (torch.ops.ewvit.linear.default, (x, w, None, 0, 0.0, 0, None, torch.float32, True, False)),
        'layer_norm': (torch.ops.ewvit.layer_norm.default, (x, _rand(64, rg=True), _rand(64, rg=True), 1e-5,
                                                            torch.float32)),
        'attention_packed': (torch.ops.ewvit.attention.default, (qkv, None, 4, 16, 0.25)),
        'attention_cross': (torch.ops.ewvit.attention.default, (q, kv, 4, 16, 0.25)),
        'dwt_haar': (torch.ops.ewvit.dwt_haar.default, (frames, 2, torch.float32)),
        'hf_upsample': (torch.ops.ewvit.hf_upsample.default, (yh, 2, 3, 32, 32, 2, 16, 16, torch.bfloat16, 16)),
    }


@pytest.mark.parametrize('name', ['linear', 'linear_gelu', 'linear_fp8', 'layer_norm', 'attention_packed',
                                  'attention_cross', 'dwt_haar', 'hf_upsample'])
def test_opcheck(name):
    op, args = _cases()[name]
    utils = ('test_schema', 'test_autograd_registration', 'test_faketensor', 'test_aot_dispatch_dynamic')
    torch.library.opcheck(op, args, test_utils=utils)


def _close(a, b):
    torch.testing.assert_close(a.float(), b.float(), rtol=1e-5, atol=1e-5)


def test_compile_vit_block_fullgraph(monkeypatch):
    # eager on the same custom ops the compiled graph holds (not the fused layer of ewvit.vit,
    # which the traced forward does not take)
    monkeypatch.setenv('EWVIT_VIT_FUSED', '0')
    from network import sfe
    torch.manual_seed(0)
    m = sfe.Transformer(512, 1, 8, 64, 2048, 0.0).to(DEV)
    cm = torch.compile(m, backend='aot_eager', fullgraph=True)
    x = torch.randn(16, 2, 512, device=DEV)
    xe, xc = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ye, yc = m(xe), cm(xc)
    _close(yc, ye)
    ye.square().sum().backward()
    ge = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    yc.square().sum().backward()
    _close(xc.grad, xe.grad)
    for n, p in m.named_parameters():
        _close(p.grad, ge[n])


def test_compile_cross_attention_fullgraph():
    from network import dama
    torch.manual_seed(1)
    m = dama.BidirectionalCrossTransformer(128, 1, 4, 32, 0.0).to(DEV)
    cm = torch.compile(m, backend='aot_eager', fullgraph=True)
    s, f = torch.randn(16, 1, 128, device=DEV), torch.randn(16, 1, 128, device=DEV)
    so, fo = m(s, f)
    sc, fc = cm(s, f)
    _close(sc, so)
    _close(fc, fo)
