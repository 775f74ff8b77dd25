"""hf_conv['fusion']'s BatchNorm + ReLU folded into multiscale_fusion's conv (reference
network/mwt.py:60-72,87-88,112-114; ewvit.conv.BnReluConvFn): the windowed forward and weight-
gradient kernels apply relu(z * scale + shift) while staging their input windows, so the
normalised 3-level map is never written.

The fold runs the same arithmetic in the same order as the two-node path (ewvit_bn_fwd_partials
apply pass, then the conv), so the whole MWT — output, every parameter gradient, every BN
running statistic and counter — must be BIT-IDENTICAL with network.mwt._FOLD_FUSION_BN off;
and the fold must actually run (ewvit_conv2d_fwd_bn_xf / ewvit_conv2d_bwd_weight_xf launched,
the fusion BN's apply pass not).  Plus the C-ABI kernels on their own against the explicit
transform: levels 1 and 3, maps of several 16 x 16 blocks with image borders on every side, a
persistent walk under a grid cap."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('hw,frames,dim', [(224, 2, 128), (64, 4, 128)])
def test_mwt_fold_bit_identical(hw, frames, dim, monkeypatch):
    import ewvit
    from network import mwt as M
    # the fusion BN's backward sums: at these sizes the two-node path would take them from the
    # multiscale conv's input-gradient epilogue (ewvit.bn BwdStatsLink, another summation order);
    # at the model's size (> BWD_LINK_MAX_ROWS tiles) it runs ewvit_bn_bwd, as the fold always does
    monkeypatch.setattr(ewvit.bn, '_BWD_LINK', False)
    monkeypatch.setattr(ewvit.conv, '_BN_BWD_EPI', False)
    torch.manual_seed(11)
    a = M.MWT(3, dim, 3).to(DEV).to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    x = torch.randn(frames, 3, hw, hw, device=DEV)
    names = []
    real = ewvit._lib.call
    monkeypatch.setattr(ewvit._lib, 'call', lambda n, *r, **k: (names.append(n), real(n, *r, **k))[1])
    with torch.autocast('cuda', dtype=torch.bfloat16):
        ya = a(x)
    ya.float().square().mean().backward()
    torch.cuda.synchronize()
    assert 'ewvit_conv2d_fwd_bn_xf' in names and 'ewvit_conv2d_bwd_weight_xf' in names and 'ewvit_bn_coef' in names
    n_apply = names.count('ewvit_bn_fwd_partials')
    names.clear()
    monkeypatch.setattr(M, '_FOLD_FUSION_BN', False)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        yb = b(x)
    yb.float().square().mean().backward()
    torch.cuda.synchronize()
    assert 'ewvit_conv2d_fwd_bn_xf' not in names
    assert names.count('ewvit_bn_fwd_partials') == n_apply + 1      # the fusion BN's apply pass
    assert torch.equal(ya, yb)
    for (n, u), v in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(u, v), n
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        if p.grad is None:
            assert q.grad is None, n
            continue
        assert torch.equal(p.grad, q.grad), n


@pytest.mark.parametrize('N,C,H,W,Cout,levels,cap', [
    (2, 128, 32, 48, 128, 3, 0),      # multiscale shape class: level-major z read as 384 channels
    (1, 64, 48, 32, 128, 1, 0),       # plain input, one channel block
    (2, 128, 32, 32, 128, 2, 5),      # 2 levels, persistent walk under a grid cap
])
def test_xf_kernels_match_explicit_transform(N, C, H, W, Cout, levels, cap):
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    from ewvit.conv import _pack
    lib = L.load()
    g = torch.Generator().manual_seed(C + H + levels)
    NL, Cx = N * levels, C * levels
    z = torch.randn(NL, C, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    coef = torch.stack([torch.rand(levels, C, generator=g) + 0.5, torch.randn(levels, C, generator=g) * 0.5], 1)
    coef = coef.to(DEV).contiguous()                    # [levels][2][C]
    # the explicit transform, bf16-rounded as the apply pass writes it (float64: one rounding, as
    # the kernel's fmaf; the float64 -> float32 -> bf16 double rounding is vanishingly rare and
    # would show as a failure of the y comparison, not pass silently)
    zl = z.double().view(levels, N, C, H, W)
    cd = coef.double()
    a = torch.relu(zl * cd[:, 0].view(levels, 1, C, 1, 1) + cd[:, 1].view(levels, 1, C, 1, 1)).float()
    a = a.view(NL, C, H, W).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cx, 3, 3, generator=g) / (9 * Cx) ** 0.5).to(DEV)
    bias = torch.randn(Cout, generator=g).to(DEV)
    wp, wpt = _pack(w, Cx, True, True)
    dy = torch.randn(N, Cout, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gc, gs = C, N * H * W * C
    assert lib.ewvit_conv2d_xf_ok(N, H, W, Cx, Cout, 3, 1, gc, gs) == 1
    shift = torch.zeros(Cout, device=DEV)
    rows = N * H * W // 256
    prev = lib.ewvit_set_grid_cap(cap)
    try:
        out = {}
        for mode in ('xf', 'ref'):
            y = torch.empty((N, Cout, H, W), dtype=torch.bfloat16, device=DEV, memory_format=torch.channels_last)
            part = torch.zeros(rows, 2 * Cout, device=DEV)
            so = torch.empty(Cout, device=DEV)
            dw = torch.empty(Cout, Cx, 3, 3, device=DEV)
            db = torch.empty(Cout, device=DEV)
            ws = torch.empty(int(lib.ewvit_conv2d_bwd_weight_workspace(N, H, W, Cx, Cout, 3, 1)) // 4, device=DEV)
            if mode == 'xf':
                L.call('ewvit_conv2d_fwd_bn_xf', L.ptr(z), L.ptr(wp), L.ptr(bias), L.ptr(y), N, H, W, Cx, Cout, gc, gs,
                       L.ptr(coef), L.ptr(shift), L.ptr(part), L.ptr(so), L.stream(y))
                L.call('ewvit_conv2d_bwd_weight_xf', L.ptr(z), L.ptr(dy), L.ptr(dw), L.ptr(db), 0, N, H, W, Cx, Cout, gc,
                       gs, L.ptr(coef), Cx, dw.stride(0), dw.stride(1), dw.stride(3), L.ptr(ws), L.stream(y))
            else:
                L.call('ewvit_conv2d_fwd_bn', L.ptr(a), L.ptr(wp), L.ptr(bias), L.ptr(y), N, H, W, Cx, Cout, 3, 1, gc,
                       gs, L.ptr(shift), L.ptr(part), L.ptr(so), L.stream(y))
                L.call('ewvit_conv2d_bwd_weight', L.ptr(a), L.ptr(dy), L.ptr(dw), L.ptr(db), 0, N, H, W, Cx, Cout, 3, 1,
                       gc, gs, Cx, dw.stride(0), dw.stride(1), dw.stride(3), L.ptr(ws), L.stream(y))
            torch.cuda.synchronize()
            out[mode] = (y, part, dw, db)
    finally:
        lib.ewvit_set_grid_cap(prev)
    for u, v, n in zip(out['xf'], out['ref'], ('y', 'bn partials', 'dW', 'db')):
        assert torch.equal(u, v), n


def test_bn_coef_matches_apply_pass():
    """ewvit_bn_coef leaves the running statistics, counter and saved mean / invstd of the apply
    pass (ewvit_bn_fwd_partials), and relu(x * scale + shift) rounded to bf16 IS that pass's output."""
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    g = torch.Generator().manual_seed(3)
    groups, M, C, nrc = 3, 3 * 4096, 128, 64
    x = torch.randn(M, C, generator=g).to(DEV, torch.bfloat16)
    xg = x.float().view(groups, nrc, M // groups // nrc, C)
    shifts = (torch.randn(groups, C, generator=g) * 0.1).to(DEV)
    d = xg - shifts.view(groups, 1, 1, C)
    part = torch.cat([d.sum(2), (d * d).sum(2)], -1).contiguous()      # [groups][nrc][2C]
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    res = {}
    for mode in ('coef', 'apply'):
        rm = torch.zeros(C, device=DEV)
        rv = torch.ones(C, device=DEV)
        cnt = torch.zeros((), dtype=torch.int64, device=DEV)
        mean = torch.empty(groups, C, device=DEV)
        inv = torch.empty(groups, C, device=DEV)
        if mode == 'coef':
            coef = torch.empty(groups, 2, C, device=DEV)
            L.call('ewvit_bn_coef', M, C, L.ptr(gamma), L.ptr(beta), L.ptr(rm), L.ptr(rv), 0.1, 1e-5, L.ptr(mean),
                   L.ptr(inv), L.ptr(cnt), L.ptr(part), L.ptr(shifts), nrc, groups, L.ptr(coef), L.stream(x))
            # (float64: the kernel's fmaf rounds once; a double rounding here is vanishingly rare)
            xl = x.double().view(groups, M // groups, C)
            cd = coef.double()
            y = torch.relu(xl * cd[:, 0].view(groups, 1, C) + cd[:, 1].view(groups, 1, C)).float().to(torch.bfloat16)
        else:
            y = torch.empty_like(x)
            L.call('ewvit_bn_fwd_partials', L.ptr(x), L.ptr(y), L.dt(x), M, C, L.ptr(gamma), L.ptr(beta), L.ptr(rm),
                   L.ptr(rv), 0.1, 1e-5, 1, L.ptr(mean), L.ptr(inv), L.ptr(cnt), L.ptr(part), L.ptr(shifts), nrc,
                   groups, L.stream(x))
        torch.cuda.synchronize()
        res[mode] = (y.view(M, C), rm, rv, cnt, mean, inv)
    assert int((res['coef'][0] != res['apply'][0]).sum()) <= 2
    for u, v, n in zip(res['coef'][1:], res['apply'][1:], ('running_mean', 'running_var', 'counter', 'mean', 'invstd')):
        assert torch.equal(u, v), n


@pytest.mark.parametrize('hw,frames', [(224, 2), (224, 32)])
def test_mwt_fold_bwd_sums_in_dgrad_epilogue(hw, frames, monkeypatch):
    """The fold with the fusion BN's backward sums taken by multiscale_fusion's windowed input-
    gradient epilogue (ewvit_conv2d_bwd_data_bn_win + ewvit_bn_bwd_partials) against its own
    reduction pass (ewvit_bn_bwd): forward and BN state identical; gradients equal up to the fp32
    summation order of those sums (cosine >= 0.99999, norms within 1e-4, and element-wise
    max |d| <= 2^-7 max |ref| — 32 frames: the model's 3 x 32 x 112^2 level maps, the default
    path of the config-2 step; the gradients of biases feeding a train-mode BN are exact zeros
    up to rounding noise and are skipped)."""
    import ewvit
    from network import mwt as M
    torch.manual_seed(12)
    a = M.MWT(3, 128, 3).to(DEV).to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    x = torch.randn(frames, 3, hw, hw, device=DEV)
    names = []
    real = ewvit._lib.call
    monkeypatch.setattr(ewvit._lib, 'call', lambda n, *r, **k: (names.append(n), real(n, *r, **k))[1])
    with torch.autocast('cuda', dtype=torch.bfloat16):
        ya = a(x)
    ya.float().square().mean().backward()
    torch.cuda.synchronize()
    assert 'ewvit_conv2d_bwd_data_bn_win' in names
    monkeypatch.setattr(ewvit.conv, '_BN_BWD_EPI', False)
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
        if n.endswith('0.bias') and not n.startswith('freq_pool'):
            continue
        u, v = p.grad.double().flatten(), q.grad.double().flatten()
        c = float(u @ v / (u.norm() * v.norm() + 1e-300))
        r = float(u.norm() / (v.norm() + 1e-300))
        e = float((u - v).abs().max() / (v.abs().max() + 1e-300))
        assert c >= 0.99999 and abs(r - 1) <= 1e-4 and e <= 2 ** -7, (n, c, r, e)


@pytest.mark.parametrize('C,Cout', [(128, 128), (128, 256)])
def test_dgrad_bn_sums_match_explicit(C, Cout):
    """ewvit_conv2d_bwd_data_bn_win: dx bit-identical to the plain windowed dgrad, the per-block
    sums of g and g * xhat equal the float64 sums over the returned dx (1e-5 of scale); Cout 256:
    4 K blocks of dy per column tile."""
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    from ewvit.conv import _pack
    lib = L.load()
    g = torch.Generator().manual_seed(21)
    N, H, W, levels = 2, 32, 48, 3
    NL, Cx = N * levels, C * levels
    gc, gs = C, N * H * W * C
    rows = int(lib.ewvit_conv2d_bwd_bn_win_rows(N, H, W, Cx, Cout, 3, 1, gc, gs, 0))
    assert rows == N * H * W // 256
    w = (torch.randn(Cout, Cx, 3, 3, generator=g) / (9 * Cx) ** 0.5).to(DEV)
    _, wpt = _pack(w, Cx, True, True)
    dy = torch.randn(N, Cout, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    z = torch.randn(NL, C, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    mean = (torch.randn(levels, C, generator=g) * 0.1).to(DEV)
    inv = (torch.rand(levels, C, generator=g) + 0.5).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    dx0 = torch.empty_like(z)
    dx1 = torch.empty_like(z)
    part = torch.full((levels * rows, 2 * C), float('nan'), device=DEV)
    L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx0), N, H, W, Cx, Cout, 3, 1, gc, gs, L.stream(dy))
    L.call('ewvit_conv2d_bwd_data_bn_win', L.ptr(dy), L.ptr(wpt), L.ptr(dx1), N, H, W, Cx, Cout, gc, gs, L.ptr(z),
           L.ptr(mean), L.ptr(inv), L.ptr(gamma), L.ptr(beta), 1, 0, L.ptr(part), L.stream(dy))
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    zl = z.double().view(levels, N, C, H, W)
    xh = (zl - mean.double().view(levels, 1, C, 1, 1)) * inv.double().view(levels, 1, C, 1, 1)
    pre = xh * gamma.double().view(1, 1, C, 1, 1) + beta.double().view(1, 1, C, 1, 1)
    gg = dx1.double().view(levels, N, C, H, W) * (pre > 0)
    # per level and 16 x 16 block (image-major, block rows, block columns)
    def blocks(t):
        return t.view(levels, N, C, H // 16, 16, W // 16, 16).sum((4, 6)).permute(0, 1, 3, 4, 2).reshape(levels, rows, C)
    s1, s2 = blocks(gg), blocks(gg * xh)
    got = part.double().view(levels, rows, 2, C)
    sc = float(s1.abs().max())
    assert float((got[:, :, 0] - s1).abs().max()) <= 1e-5 * sc
    sc2 = float(s2.abs().max())
    assert float((got[:, :, 1] - s2).abs().max()) <= 1e-5 * sc2


@pytest.mark.parametrize('cap', [0, 5])
def test_dgrad_bn_sums_row_groups_ksplit(cap):
    """The k-split 64-column input gradient (hf_conv['fusion'] 128 -> 64) with BatchNorm ROW
    groups (the seperate BNs' per-level statistics: slices of whole images): dx bit-identical to
    the plain windowed dgrad, part [levels][blocks per level][2 C] equal to the float64 sums
    over the returned dx with each level's own mean / invstd (1e-5 of scale); cap 5: the
    persistent walk."""
    import ewvit  # noqa: F401
    from ewvit import _lib as L
    from ewvit.conv import _pack
    lib = L.load()
    g = torch.Generator().manual_seed(23 + cap)
    levels, N, C, H, W, Cout = 3, 2, 64, 32, 48, 128
    NL = levels * N
    grows = N * H * W
    rows = int(lib.ewvit_conv2d_bwd_bn_win_rows(NL, H, W, C, Cout, 3, 1, C, 0, grows))
    assert rows == NL * H * W // 256
    assert int(lib.ewvit_conv2d_bwd_bn_win_rows(NL, H, W, C, Cout, 3, 1, C, 0, grows // 2 + 256)) == 0   # not whole images
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(DEV)
    _, wpt = _pack(w, C, True, True)
    dy = torch.randn(NL, Cout, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    z = torch.randn(NL, C, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    mean = (torch.randn(levels, C, generator=g) * 0.1).to(DEV)
    inv = (torch.rand(levels, C, generator=g) + 0.5).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    dx0 = torch.empty_like(z)
    dx1 = torch.empty_like(z)
    part = torch.full((rows, 2 * C), float('nan'), device=DEV)
    prev = lib.ewvit_set_grid_cap(cap)
    try:
        L.call('ewvit_conv2d_bwd_data', L.ptr(dy), L.ptr(wpt), L.ptr(dx0), NL, H, W, C, Cout, 3, 1, 0, 0, L.stream(dy))
        L.call('ewvit_conv2d_bwd_data_bn_win', L.ptr(dy), L.ptr(wpt), L.ptr(dx1), NL, H, W, C, Cout, C, 0, L.ptr(z),
               L.ptr(mean), L.ptr(inv), L.ptr(gamma), L.ptr(beta), 1, grows, L.ptr(part), L.stream(dy))
        torch.cuda.synchronize()
    finally:
        lib.ewvit_set_grid_cap(prev)
    assert torch.equal(dx0, dx1)
    dref = torch.nn.grad.conv2d_input(z.shape, w.to(torch.bfloat16).float(), dy.float(), padding=1)
    assert float((dx1.float() - dref).abs().max() / dref.abs().max()) < 2 ** -7
    zl = z.double().view(levels, N, C, H, W)
    xh = (zl - mean.double().view(levels, 1, C, 1, 1)) * inv.double().view(levels, 1, C, 1, 1)
    pre = xh * gamma.double().view(1, 1, C, 1, 1) + beta.double().view(1, 1, C, 1, 1)
    gg = dx1.double().view(levels, N, C, H, W) * (pre > 0)
    nb = rows // levels

    def blocks(t):
        return t.view(levels, N, C, H // 16, 16, W // 16, 16).sum((4, 6)).permute(0, 1, 3, 4, 2).reshape(levels, nb, C)
    s1, s2 = blocks(gg), blocks(gg * xh)
    got = part.double().view(levels, nb, 2, C)
    assert float((got[:, :, 0] - s1).abs().max()) <= 1e-5 * float(s1.abs().max())
    assert float((got[:, :, 1] - s2).abs().max()) <= 1e-5 * float(s2.abs().max())
