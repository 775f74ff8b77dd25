"""The hot-path ops are torch.library custom ops (torch.ops.ewvit.*) with fake
(meta) implementations: FakeTensor tracing and make_fx see them as single ops without
launching kernels — no GPU needed for these checks (the GPU tests run the real kernels, and
test_gpu_custom_ops.py runs torch.library.opcheck and torch.compile on them)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode
from torch.fx.experimental.proxy_tensor import make_fx

OPS = ['linear', 'linear_backward', 'layer_norm', 'layer_norm_backward', 'attention', 'attention_backward',
       'dwt_haar', 'hf_upsample']


def test_ops_registered_with_schemas():
    import ewvit  # noqa: F401  (registers the ops)
    for name in OPS:
        op = getattr(torch.ops.ewvit, name)
        assert op.default._schema.name == f'ewvit::{name}'
    assert 'Tensor(a' in str(torch.ops.ewvit.linear_backward.default._schema)   # dw_out / db_out mutated


@pytest.mark.parametrize('dev', ['cuda', 'cpu'])
def test_fake_tensor_forward_backward_shapes(dev):
    """Fake 'cuda' tensors trace the forward on this GPU-less host; the autograd engine needs
    a real device context for cuda, so the backward is traced on fake 'cpu' tensors (the fake
    implementations are device-agnostic)."""
    import ewvit
    with FakeTensorMode():
        x = torch.empty(64, 2, 512, device=dev, requires_grad=True)
        w1 = torch.empty(1536, 512, device=dev, requires_grad=True)
        g = torch.empty(512, device=dev, requires_grad=True)
        b = torch.empty(512, device=dev, requires_grad=True)
        h = ewvit.layer_norm(x, g, b, 1e-5, out_dtype=torch.bfloat16)
        qkv = ewvit.linear(h, w1, None, out_dtype=torch.bfloat16)
        o = ewvit.attention_packed(qkv, 8, 64, 0.125)
        w2 = torch.empty(512, 512, device=dev, requires_grad=True)
        y = ewvit.linear(o, w2, None, act=1, out_dtype=torch.float32, fp8=True)
        assert y.shape == (64, 2, 512) and y.dtype == torch.float32
        if dev == 'cpu':
            y.sum().backward()
            assert x.grad.shape == x.shape and w1.grad.shape == w1.shape and w2.grad.shape == w2.shape
            assert g.grad.shape == (512,)
        frames = torch.empty(4, 3, 224, 224, device=dev)
        up, ll = ewvit.dwt_hf_upsample(frames, 3, (112, 112), out_channels=16)
        assert up.shape == (3, 4, 112, 112, 16) and ll.shape == (4, 3, 28, 28)
        ll1, yh = ewvit.dwt_haar(frames, 2)
        assert [t.shape for t in yh] == [(4, 3, 3, 112, 112), (4, 3, 3, 56, 56)]


def test_make_fx_traces_ops_as_single_nodes():
    import ewvit

    def f(x, w, b, g, beta):
        h = ewvit.layer_norm(x, g, beta, 1e-5, out_dtype=torch.bfloat16)
        return ewvit.linear(h, w, b, act=2, out_dtype=torch.float32)
    args = (torch.randn(8, 2, 64), torch.randn(32, 64), torch.randn(32), torch.randn(64), torch.randn(64))
    gm = make_fx(f, tracing_mode='fake')(*args)
    targets = [str(n.target) for n in gm.graph.nodes if n.op == 'call_function']
    assert 'ewvit.layer_norm.default' in targets and 'ewvit.linear.default' in targets
    assert not any('addmm' in t or 'native_layer_norm' in t for t in targets)


def test_real_implementation_refuses_cpu():
    import ewvit
    if not ewvit._lib.os.path.exists(ewvit._lib.LIB_PATH):
        pytest.skip('library not built')
    with pytest.raises(RuntimeError, match='MI355X only'):
        ewvit.linear(torch.randn(4, 8), torch.randn(6, 8))
