"""Deferred weight-gradient reductions (csrc/reduce_jobs.h, ewvit/defer.py): a deferred
split-K / depthwise slab reduce that runs in front of a later weight-gradient launch, or in
the end-of-backward flush, gives the SAME bits as the immediate reduce launch (same code,
same summation order), on the library entry points and on the backbone's MBConv stages in a
training step (eager and HIP-graph replay)."""
import copy
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _lib():
    import ewvit
    return ewvit._lib


def _wgrad(x, dy, k, defer, N, H, W, Cin, Cout):
    """dW of a k x k conv via ewvit_conv2d_bwd_weight; (dW, workspace) — the workspace must
    outlive a deferred job."""
    L = _lib()
    lib = L.load()
    wsb = lib.ewvit_conv2d_bwd_weight_workspace(N, H, W, Cin, Cout, k, 1)
    ws = torch.empty(wsb // 4, dtype=torch.float32, device=DEV)
    dw = torch.full((Cout, Cin, k, k), float('nan'), dtype=torch.float32, device=DEV)
    if defer:
        lib.ewvit_reduce_defer_next(1)
    s = dw.stride()
    L.call('ewvit_conv2d_bwd_weight', L.ptr(x), L.ptr(dy), L.ptr(dw), None, 0, N, H, W, Cin, Cout, k, 1, 0, 0,
           Cin, s[0], s[1], s[3], L.ptr(ws), L.stream(dw))
    return dw, ws


def _pending():
    return int(_lib().load().ewvit_reduce_pending(None))


@pytest.mark.parametrize('shapes', [
    # (N, H, W, Cin, Cout, k): stage-6 expand / project 1x1, a FusedMBConv 3x3, ragged pixels
    [(64, 7, 7, 256, 1536, 1), (64, 7, 7, 1536, 256, 1), (8, 28, 28, 48, 64, 3)],
    [(8, 28, 28, 64, 256, 1), (6, 13, 11, 64, 64, 3), (3, 11, 13, 128, 512, 1)],
])
def test_deferred_reduce_bit_exact(shapes):
    """Each wgrad deferred; every later one hosts the earlier jobs; the flush runs the last."""
    g = torch.Generator(device=DEV).manual_seed(7)
    ops = []
    for (N, H, W, Cin, Cout, k) in shapes:
        x = torch.randn(N, H, W, Cin, device=DEV, generator=g).to(torch.bfloat16)
        dy = torch.randn(N, H, W, Cout, device=DEV, generator=g).to(torch.bfloat16)
        ops.append((x, dy, k, N, H, W, Cin, Cout))
    ref = [_wgrad(x, dy, k, False, N, H, W, Cin, Cout)[0] for (x, dy, k, N, H, W, Cin, Cout) in ops]
    torch.cuda.synchronize()
    assert _pending() == 0
    outs, keep, queued = [], [], []
    for i, (x, dy, k, N, H, W, Cin, Cout) in enumerate(ops):
        dw, ws = _wgrad(x, dy, k, True, N, H, W, Cin, Cout)
        outs.append(dw)
        keep.append(ws)
        queued.append(_pending())               # (a one-split call writes dW directly: nothing queued)
    assert queued[0] == 1 and max(queued) >= 1, queued
    lib = _lib().load()
    assert lib.ewvit_reduce_flush(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    assert _pending() == 0
    torch.cuda.synchronize()
    for a, b in zip(outs, ref):
        assert not torch.isnan(a).any()
        assert torch.equal(a, b)


def test_defer_mark_consumed_by_next_call():
    """The mark applies to exactly one call: a windowed / biased call consumes it without
    queueing, and the call after it reduces immediately."""
    lib = _lib().load()
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(4, 14, 14, 64, device=DEV, generator=g).to(torch.bfloat16)
    dy = torch.randn(4, 14, 14, 128, device=DEV, generator=g).to(torch.bfloat16)
    lib.ewvit_reduce_defer_next(1)
    L = _lib()
    wsb = lib.ewvit_conv2d_bwd_weight_workspace(4, 14, 14, 64, 128, 1, 1)
    ws = torch.empty(wsb // 4, dtype=torch.float32, device=DEV)
    dw = torch.empty(128, 64, 1, 1, device=DEV)
    db = torch.empty(128, device=DEV)
    s = dw.stride()
    L.call('ewvit_conv2d_bwd_weight', L.ptr(x), L.ptr(dy), L.ptr(dw), L.ptr(db), 0, 4, 14, 14, 64, 128, 1, 1, 0, 0,
           64, s[0], s[1], s[3], L.ptr(ws), L.stream(dw))
    assert _pending() == 0                      # bias gradient: never deferred
    dw2, _ = _wgrad(x, dy, 1, False, 4, 14, 14, 64, 128)
    assert _pending() == 0
    torch.cuda.synchronize()
    # (the biased call takes the generic kernel, the unbiased one the 1x1 kernel: other splits)
    torch.testing.assert_close(dw, dw2, rtol=1e-5, atol=1e-4)


class _NoOpt:
    def __init__(self, params):
        self.params = list(params)
        self.param_groups = [{'params': self.params}]

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def step(self):
        pass


def _stages():
    from network.efficientnet import EfficientNetV2S
    torch.manual_seed(11)
    net = EfficientNetV2S()
    # stages 3-6 (FusedMBConv 48 -> 64, MBConv 64 -> 128 -> 160 -> 256) and the 1x1 head
    m = torch.nn.Sequential(*list(net.features.children())[3:]).to(DEV).to(memory_format=torch.channels_last)
    return m.train()


def _grads(m, x, graph, enabled, steps=1):
    import ewvit
    from ewvit import defer
    from ewvit.graph import TrainStep
    calls = []
    real = defer.mark

    def spy(ws, out, dev):
        ok = real(ws, out, dev)
        calls.append(ok)
        return ok
    old, defer.ENABLED, defer.mark = defer.ENABLED, enabled, spy
    try:
        def fl():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                return m(x).float().square().mean()
        torch.manual_seed(5)
        st = TrainStep(m, fl, _NoOpt(p for p in m.parameters() if p.requires_grad), graph=graph, warmup=2)
        for _ in range(steps):
            torch.manual_seed(5)
            st()
        torch.cuda.synchronize()
        out = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        st.close()
    finally:
        defer.ENABLED, defer.mark = old, real
    assert _pending() == 0
    del ewvit
    return out, sum(calls)


@pytest.mark.parametrize('graph', [False, True])
def test_backbone_stages_bit_exact(graph):
    """MBConv / FusedMBConv stages in a TrainStep: the gradients with deferral equal the
    gradients without, bit for bit, and the deferral is actually taken."""
    a = _stages()
    b = copy.deepcopy(a)
    x = torch.randn(8, 48, 56, 56, device=DEV).to(memory_format=torch.channels_last)
    ga, na = _grads(a, x, graph, False)
    gb, nb = _grads(b, x, graph, True)
    assert na == 0 and nb > 40, (na, nb)
    assert ga.keys() == gb.keys() and len(ga) > 100
    for n in ga:
        assert torch.equal(ga[n], gb[n]), n


def _stage_grads(m, x, graph, **switches):
    """Parameter gradients and the input gradient of `m` on x after one TrainStep, with module
    switches set for the duration (module, attribute) -> value."""
    from ewvit.graph import TrainStep
    old = {k: getattr(k[0], k[1]) for k in switches.get('sw', {})}
    try:
        for (mod, attr), v in switches.get('sw', {}).items():
            setattr(mod, attr, v)
        xi = x.clone().requires_grad_(True)

        def fl():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                return m(xi).float().square().mean()
        torch.manual_seed(5)
        st = TrainStep(m, fl, _NoOpt(p for p in m.parameters() if p.requires_grad), graph=graph, warmup=2)
        torch.manual_seed(5)
        st()
        torch.cuda.synchronize()
        out = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        out['__x__'] = xi.grad.clone()
        st.close()
    finally:
        for (mod, attr), v in old.items():
            setattr(mod, attr, v)
    return out


@pytest.mark.parametrize('graph', [False, True])
def test_se_dx_fold(graph):
    """MBConv's depthwise BN + SE backward with its dx pass folded into the depthwise conv's
    fused backward (ewvit.se.SeDxLink, ewvit_dwconv3x3_bwd_fused_se; an A/B option, off by
    default) against the separate dx pass: the fold is taken in the stride-1 blocks and the
    gradients agree to bf16 rounding (dz may differ by one rounding with SiLU, which the
    backward through 30 blocks spreads: relative L2 error of all gradients < 5e-2); the fallback
    that materialises the dx pass when the conv cannot fold gives the same bits."""
    import ewvit.ops as eops
    import ewvit.se as ese
    a = _stages()
    # (copies before any step: the BatchNorm statistics are summed centred on the running mean)
    b, c, d = copy.deepcopy(a), copy.deepcopy(a), copy.deepcopy(a)
    x = torch.randn(8, 48, 56, 56, device=DEV).to(memory_format=torch.channels_last)
    calls = []
    real = ese.SeDxLink.take

    def spy(self):
        calls.append(1)
        return real(self)
    ga = _stage_grads(a, x, graph, sw={(ese, '_SE_DX_FOLD'): False})
    ese.SeDxLink.take = spy
    try:
        gb = _stage_grads(b, x, graph, sw={(ese, '_SE_DX_FOLD'): True})
    finally:
        ese.SeDxLink.take = real
    assert len(calls) >= 20, len(calls)              # the stride-1 MBConv blocks fold
    # the fold refused by the conv (its fused backward off): the dx pass materialised
    gc = _stage_grads(c, x, graph, sw={(ese, '_SE_DX_FOLD'): True, (eops, '_DW_BWD_FUSED'): False})
    gd = _stage_grads(d, x, graph, sw={(ese, '_SE_DX_FOLD'): False, (eops, '_DW_BWD_FUSED'): False})
    assert ga.keys() == gb.keys() and len(ga) > 100
    va = torch.cat([ga[n].flatten() for n in ga])
    vb = torch.cat([gb[n].flatten() for n in ga])
    assert float((va - vb).norm() / va.norm()) < 5e-2        # (measured 1.6e-2)
    dcd = [n for n in gd if not torch.equal(gc[n], gd[n])]
    assert not dcd, dcd[:6]


def test_defer_after_failed_backward():
    """A backward pass that raises after deferring reductions leaves its jobs queued; the next
    backward's first deferral runs them (into memory kept alive for them) and its own gradients
    come out right — the same bits as with the deferral off."""
    import ewvit
    from ewvit import defer, grads
    from network.efficientnet import Conv2d

    class Boom(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.clone()

        @staticmethod
        def backward(ctx, g):
            raise RuntimeError('boom')

    torch.manual_seed(3)
    c1 = Conv2d(64, 256, 1, bias=False).to(DEV).to(memory_format=torch.channels_last)
    c2 = Conv2d(256, 128, 1, bias=False).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(8, 64, 28, 28, device=DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)

    def run(fail, enabled):
        old, defer.ENABLED = defer.ENABLED, enabled
        try:
            for p in (*c1.parameters(), *c2.parameters()):
                p.grad = None
            grads.begin_step()
            h = c1(x)
            y = c2(Boom.apply(h) if fail else h)
            loss = y.float().square().mean()
            if fail:
                with pytest.raises(RuntimeError, match='boom'):
                    loss.backward()
            else:
                loss.backward()
            grads.end_step()
        finally:
            defer.ENABLED = old
        return c1.weight.grad, c2.weight.grad

    ref = [g.clone() for g in run(False, False)]
    calls = []
    real = defer.mark
    defer.mark = lambda ws, out, dev: calls.append(1) or real(ws, out, dev)
    try:
        run(True, True)                                  # c2's wgrad deferred, then the raise
        assert calls and _pending() >= 1
        got = run(False, True)
    finally:
        defer.mark = real
    torch.cuda.synchronize()
    assert _pending() == 0
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
