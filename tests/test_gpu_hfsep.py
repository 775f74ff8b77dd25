"""The MWT seperate convs on csrc/hfsep.hip (reference network/mwt.py:48-59, 84-86: three
Conv2d(3, 18, 3, pad 1), colour g's three HF bands each, weights shared by the levels) against
torch fp32 on the same bf16-rounded operands.

Bounds: forward output within one bf16 rounding of the fp32 result (the kernel rounds the
weights to bf16 — the MFMA operand type — and rounds its fp32 sum once); the BatchNorm partial
sums equal the sums of the kernel's own bf16 output to 1e-5 of scale (fp32 summation order);
weight / bias gradients from bf16 x and dy with fp32 accumulation equal the fp32 reference to
2e-4 of scale (summation order over up to 2.4 M pixels)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _convs(seed):
    torch.manual_seed(seed)
    return [torch.nn.Conv2d(3, 18, 3, padding=1).to(DEV) for _ in range(3)]


def _input(L, N, H, W, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.zeros(L * N, H, W, 16, device=DEV, dtype=torch.bfloat16)
    x[..., :9] = torch.randn(L * N, H, W, 9, device=DEV, generator=g).to(torch.bfloat16)
    return x.permute(0, 3, 1, 2)                       # NCHW view of NHWC memory


def _ref_fwd(x, convs):
    xf = x.float()
    outs = [F.conv2d(xf[:, 3 * i:3 * i + 3], c.weight.detach().to(torch.bfloat16).float(), c.bias.detach(), padding=1)
            for i, c in enumerate(convs)]
    return torch.cat(outs, 1)


@pytest.mark.parametrize('L,N,H,W', [(3, 2, 32, 32), (1, 1, 112, 112), (3, 1, 20, 28), (2, 2, 9, 13)])
def test_seperate_forward_and_bn_partials(L, N, H, W):
    import ewvit
    convs = _convs(1)
    x = _input(L, N, H, W, 2)
    shift = torch.randn(64, device=DEV) * 0.1
    shift[54:] = 0
    y, (part, shifts, nrc) = ewvit.hfsep.seperate_conv(x, L, convs, shift=shift)
    torch.cuda.synchronize()
    assert y.shape == (L * N, 64, H, W) and y.is_contiguous(memory_format=torch.channels_last)
    ref = _ref_fwd(x, convs)
    yf = y.float()
    scale = ref.abs().max()
    torch.testing.assert_close(yf[:, :54], ref, rtol=0, atol=float(scale) * 2 ** -8)
    assert not yf[:, 54:].any()
    # partial statistics, per level: sum (y - K) and sum (y - K)^2 of the bf16 output
    yl = yf.view(L, N, 64, H, W)
    d = yl - shift.view(1, 1, 64, 1, 1)
    s1 = d.sum((1, 3, 4))
    s2 = (d * d).sum((1, 3, 4))
    got = part.sum(1)
    torch.testing.assert_close(got[:, :64], s1, rtol=1e-5, atol=1e-5 * float(s2.detach().max()) ** 0.5 * (N * H * W) ** 0.5)
    torch.testing.assert_close(got[:, 64:], s2, rtol=1e-5, atol=1e-4)
    assert torch.equal(shifts, shift.view(1, 64).expand(L, 64))
    assert part.shape == (L, nrc, 128) and 1 <= nrc <= 256


@pytest.mark.parametrize('L,N,H,W', [(3, 2, 32, 32), (1, 2, 112, 112), (3, 1, 20, 28), (2, 2, 9, 13)])
def test_seperate_weight_gradients(L, N, H, W):
    import ewvit
    convs = _convs(3)
    x = _input(L, N, H, W, 4)
    y = ewvit.hfsep.seperate_conv(x, L, convs)
    g = torch.Generator(device=DEV).manual_seed(5)
    dy = torch.randn(y.shape, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy[:, 54:] = 0
    y.backward(dy)
    torch.cuda.synchronize()
    xf = x.float()
    for i, c in enumerate(convs):
        w = c.weight.detach().clone().requires_grad_(True)
        b = c.bias.detach().clone().requires_grad_(True)
        out = F.conv2d(xf[:, 3 * i:3 * i + 3], w, b, padding=1)
        out.backward(dy[:, 18 * i:18 * i + 18].float())
        sw, sb = float(w.grad.abs().max()), float(b.grad.abs().max())
        torch.testing.assert_close(c.weight.grad, w.grad, rtol=0, atol=2e-4 * sw, msg=f'weight {i}')
        torch.testing.assert_close(c.bias.grad, b.grad, rtol=0, atol=2e-4 * sb, msg=f'bias {i}')


def test_seperate_capped_grid_same_results():
    """under the MWT branch's workgroup cap (ewvit._lib.grid_cap) the output is bit-identical,
    the weight gradients and statistics change only their fp32 summation order"""
    import ewvit
    convs = _convs(7)
    x = _input(3, 2, 56, 56, 8)
    shift = torch.zeros(64, device=DEV)
    y0, (p0, _, _) = ewvit.hfsep.seperate_conv(x, 3, convs, shift=shift)
    dy = torch.randn(y0.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y0.backward(dy)
    g0 = [c.weight.grad.clone() for c in convs]
    for c in convs:
        c.weight.grad = None
        c.bias.grad = None
    with ewvit._lib.grid_cap(16):
        y1, (p1, _, n1) = ewvit.hfsep.seperate_conv(x, 3, convs, shift=shift)
        y1.backward(dy)
    torch.cuda.synchronize()
    assert n1 <= 16 // 3 + 1
    assert torch.equal(y0, y1)
    torch.testing.assert_close(p1.sum(1), p0.sum(1), rtol=1e-5, atol=1e-3)
    for a, c in zip(g0, convs):
        torch.testing.assert_close(c.weight.grad, a, rtol=1e-5, atol=1e-5 * float(a.abs().max()))


def test_mwt_uses_grouped_seperate_and_matches_block_diagonal():
    """MWT._hf_features on the grouped kernel against the block-diagonal dense conv path it
    replaced and the fp32 oracle (oracle/model.py MWT, same weights and input, train mode):
    the grouped path is used, and its output and every parameter gradient are at least as
    close to the oracle as the replaced path's (cosine margin 0.02 for the bf16 noise of
    the different BatchNorm statistics summation — both paths reach only 0.95-0.96 on the
    seperate BatchNorm gammas at 4 frames per level; floors 0.9999 / 0.98)."""
    import copy
    import ewvit
    from network.mwt import MWT
    from oracle import model as om
    torch.manual_seed(11)
    a = MWT(3, 64, 3).to(DEV).to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    o = om.MWT(3, 64, 3).train()
    o.load_state_dict({k: v.detach().cpu() for k, v in a.state_dict().items()})
    x = torch.randn(4, 3, 64, 64, device=DEV)
    calls = []
    orig, orig_bn = ewvit.hfsep.SeperateConvFn.apply, ewvit.hfsep.SeperateBNReLUFn.apply

    def spy(*args):
        calls.append(1)
        return orig(*args)

    def spy_bn(*args):
        calls.append(2)
        return orig_bn(*args)
    ewvit.hfsep.SeperateConvFn.apply = spy
    ewvit.hfsep.SeperateBNReLUFn.apply = spy_bn
    try:
        with torch.autocast('cuda', dtype=torch.bfloat16):
            ya = a(x)
    finally:
        ewvit.hfsep.SeperateConvFn.apply = orig
        ewvit.hfsep.SeperateBNReLUFn.apply = orig_bn
    assert calls, 'the grouped seperate conv was not used'
    applies = ewvit.hfsep.applies
    ewvit.hfsep.applies = lambda *_: False            # the block-diagonal dense conv path
    try:
        with torch.autocast('cuda', dtype=torch.bfloat16):
            yb = b(x)
    finally:
        ewvit.hfsep.applies = applies
    yo = o(x.cpu())
    ya.float().square().mean().backward()
    yb.float().square().mean().backward()
    yo.square().mean().backward()
    torch.cuda.synchronize()

    def cos(u, v):
        return float(torch.nn.functional.cosine_similarity(u.detach().double().cpu().flatten(),
                                                            v.detach().double().cpu().flatten(), dim=0))
    assert cos(ya, yo) > 0.9999 and cos(ya, yo) >= cos(yb, yo) - 1e-4
    mods = dict(a.named_modules())
    po = dict(o.named_parameters())
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        if p.grad is None:
            continue
        if n.endswith('.bias') and isinstance(mods[n[:-5]], torch.nn.Conv2d):
            continue          # every MWT conv feeds a train-mode BN: exact zero gradient, rounding noise
        ca, cb = cos(p.grad, po[n].grad), cos(q.grad, po[n].grad)
        assert ca >= min(0.98, cb - 0.02), (n, ca, cb)
    for (n, u), v in zip(a.named_buffers(), b.buffers()):
        if u.dtype.is_floating_point:
            torch.testing.assert_close(u, v, rtol=2e-3, atol=2e-3, msg=n)
        else:
            assert torch.equal(u, v), n


@pytest.mark.parametrize('hw', [64, 224])
def test_fused_seperate_bn_node_matches_two_node_path(hw, monkeypatch):
    """SeperateBNReLUFn (the BN's dx recomputed inside the weight-gradient pass, the BN backward
    sums taken from the fusion conv's input-gradient epilogue) against the two-node path
    (SeperateConvFn + the grouped BatchNormActFn): forward bit-identical, the BN running
    statistics identical, every gradient outside the seperate conv / its BN bit-identical, and
    the seperate conv's and BN's gradients equal up to the order of fp32 operations before dy's
    bf16 rounding (cosine >= 0.99999, norms within 1e-4)."""
    import copy
    import ewvit
    from network import mwt as M
    torch.manual_seed(5)
    a = M.MWT(3, 128, 3).to(DEV).to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    x = torch.randn(4, 3, hw, hw, device=DEV)
    names = []
    real = ewvit._lib.call
    monkeypatch.setattr(ewvit._lib, 'call', lambda n, *r, **k: (names.append(n), real(n, *r, **k))[1])
    with torch.autocast('cuda', dtype=torch.bfloat16):
        ya = a(x)
    ya.float().square().mean().backward()
    assert 'ewvit_hfsep_bn_bwd_weight' in names and 'ewvit_hfsep_bwd_weight' not in names
    monkeypatch.setattr(M, '_FUSED_SEP_BN', False)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        yb = b(x)
    yb.float().square().mean().backward()
    torch.cuda.synchronize()
    assert torch.equal(ya, yb)
    for (n, u), v in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(u, v), n
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        if p.grad is None:
            assert q.grad is None, n
            continue
        if n.startswith('hf_conv.seperate.'):
            u, v = p.grad.double().flatten(), q.grad.double().flatten()
            c = float(u @ v / (u.norm() * v.norm() + 1e-300))
            r = float(u.norm() / (v.norm() + 1e-300))
            print(f'{n}: cos {c:.8f} norm ratio {r:.7f}')
            if n.endswith('0.bias'):        # feeds a train-mode BN: an exact zero, rounding noise
                continue
            assert c >= 0.99999 and abs(r - 1) <= 1e-4, (n, c, r)
        else:
            assert torch.equal(p.grad, q.grad), n


@pytest.mark.parametrize('L,N,H,W', [(3, 2, 32, 32), (1, 1, 112, 112), (2, 1, 20, 192), (1, 2, 16, 6)])
def test_nine_channel_input_bit_identical(L, N, H, W):
    """x with the 9 real band channels only (18 B per pixel; the kernels zero-pad K in LDS)
    against the 16-channel layout: forward output, BN partial sums and every weight / bias
    gradient bit-identical (the LDS images the MFMAs read are the same); W 192: the wider
    staging forms (config 4's 192-wide level maps)."""
    import ewvit
    convs = _convs(13)
    x16 = _input(L, N, H, W, 14)
    x9 = x16[:, :9].contiguous(memory_format=torch.channels_last)
    assert x9.stride(1) == 1 and x9.stride(3) == 9
    shift = torch.randn(64, device=DEV) * 0.1
    shift[54:] = 0
    g = torch.Generator(device=DEV).manual_seed(15)
    out = []
    for x in (x16, x9):
        for c in convs:
            c.weight.grad = None
            c.bias.grad = None
        y, (part, shifts, nrc) = ewvit.hfsep.seperate_conv(x, L, convs, shift=shift)
        dy = torch.randn(y.shape, device=DEV, generator=g.manual_seed(15)).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y.backward(dy)
        torch.cuda.synchronize()
        out.append((y, part, [c.weight.grad.clone() for c in convs] + [c.bias.grad.clone() for c in convs]))
    (y0, p0, g0), (y1, p1, g1) = out
    assert torch.equal(y0, y1)
    assert torch.equal(p0, p1)
    for a, b in zip(g0, g1):
        assert torch.equal(a, b)


def test_dwt_front_end_nine_channels():
    """ewvit.dwt_hf_features with 9 output channels: the first 9 channels of the 16-channel
    output, bit for bit, on the fused launch (224^2 frames) and the two-launch path (384^2)."""
    import ewvit
    for hw in (224, 384):
        x = torch.randn(2, 3, hw, hw, device=DEV)
        a = ewvit.dwt_hf_features(x, 3, (hw // 2, hw // 2), out_dtype=torch.bfloat16, out_channels=16)
        b = ewvit.dwt_hf_features(x, 3, (hw // 2, hw // 2), out_dtype=torch.bfloat16, out_channels=9)
        torch.cuda.synchronize()
        assert b.shape[-1] == 9
        assert torch.equal(a[..., :9], b), hw


@pytest.mark.parametrize('hw', [64, 224])
def test_mwt_nine_channel_front_end_bit_identical(hw, monkeypatch):
    """The MWT with the 9-channel HF layout (ewvit.hfsep.HF9) against the 16-channel one: output,
    BN state and every parameter gradient bit-identical."""
    import copy
    import ewvit
    from network import mwt as M
    torch.manual_seed(6)
    a = M.MWT(3, 128, 3).to(DEV).to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    x = torch.randn(2, 3, hw, hw, device=DEV)
    shapes = []
    real = ewvit.hfsep.applies
    monkeypatch.setattr(ewvit.hfsep, 'applies', lambda t, c: (shapes.append(t.shape[1]), real(t, c))[1])
    with torch.autocast('cuda', dtype=torch.bfloat16):
        ya = a(x)
    ya.float().square().mean().backward()
    monkeypatch.setattr(ewvit.hfsep, 'HF9', False)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        yb = b(x)
    yb.float().square().mean().backward()
    torch.cuda.synchronize()
    assert shapes == [9, 16]
    assert torch.equal(ya, yb)
    for (n, u), v in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(u, v), n
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        assert (p.grad is None) == (q.grad is None), n
        if p.grad is not None:
            assert torch.equal(p.grad, q.grad), n
