"""Capped grids (ewvit_set_grid_cap; the MWT branch runs under a cap of 160 workgroups
beside the backbone, network/dama.py:_mwt_grid_cap): the LDS-DMA convs walk their tiles
persistently with the next tile's K-tiles staged during the current tile's tail, the
register-staged conv walks its M-tiles, and BatchNorm / wgrad re-partition their rows.

A tile is computed the same way whoever walks it, so the conv outputs and input
gradients are bit-identical to the uncapped launch; weight gradients (fewer pixel
splits under a cap) and BatchNorm statistics (more rows per block) only change their
fp32 summation order: <= 1e-5 of scale.  Small caps (8, 24 workgroups) give every block
many tiles, so each walk crosses tile boundaries with K-tiles in flight."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


@pytest.fixture(params=[1, 0], ids=['glds', 'regstage'])
def variant(request):
    import ewvit
    lib = ewvit._lib.load()
    prev = lib.ewvit_conv2d_set_glds(request.param)
    yield request.param
    lib.ewvit_conv2d_set_glds(prev)


def _run_conv(x, w, b, stride, cap, dy):
    import ewvit
    import ewvit.conv as ec
    xd = x.clone().requires_grad_(True)
    wd, bd = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    with ewvit._lib.grid_cap(cap):
        y = ec.conv2d(xd, wd, bd, stride)
        y.backward(dy)
    torch.cuda.synchronize()
    return y.detach(), xd.grad, wd.grad, bd.grad


@pytest.mark.parametrize('cap', [8, 24])
@pytest.mark.parametrize('N,Cin,Cout,H,W,stride,k', [
    (4, 128, 128, 56, 56, 1, 3),     # 98 x 1 tiles, 18 K-tiles each
    (3, 64, 384, 30, 31, 1, 3),      # 3 column tiles, ragged M
    (2, 128, 128, 57, 55, 2, 3),     # stride 2: parity-class dgrad
    (5, 64, 64, 33, 35, 1, 1),       # 1x1: one K-tile per tile (walk crosses tiles every step)
    (4, 1536, 1536, 7, 7, 1, 1),     # long K, few tiles
    (2, 56, 64, 40, 40, 1, 3),       # 56 channels: the MWT fusion conv shape class
])
def test_capped_conv_matches_uncapped(N, Cin, Cout, H, W, stride, k, cap, variant):
    g = torch.Generator().manual_seed(N * Cin + H + k)
    x = torch.randn(N, Cin, H, W, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (k * k * Cin) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    Ho = (H - 1) // stride + 1
    Wo = (W - 1) // stride + 1
    dy = torch.randn(N, Cout, Ho, Wo, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    ref = _run_conv(x, w, b, stride, 0, dy)
    got = _run_conv(x, w, b, stride, cap, dy)
    assert torch.equal(got[0], ref[0])          # output: same tiles, same K order
    assert torch.equal(got[1], ref[1])          # input gradient
    assert rel(got[2], ref[2]) <= 1e-5          # weight gradient: other pixel splits
    assert rel(got[3], ref[3]) <= 1e-5


@pytest.mark.parametrize('cap', [8, 40])
@pytest.mark.parametrize('cin,cout,k,stride,hw', [(64, 256, 1, 1, 28), (128, 160, 3, 2, 29), (64, 64, 3, 1, 33)])
def test_capped_conv_bn_epilogue_stats(cin, cout, k, stride, hw, cap):
    """ConvBNAct with the BatchNorm sums in the conv epilogue (the statistics image sits
    after the LDS ring, so the next tile's K-tiles land while it is reduced)."""
    import ewvit
    from network.efficientnet import ConvBNAct
    torch.manual_seed(cin + cout + k)
    m1 = ConvBNAct(cin, cout, k, stride).to(DEV)
    m2 = ConvBNAct(cin, cout, k, stride).to(DEV)
    m2.load_state_dict(m1.state_dict())
    with torch.no_grad():
        for m in (m1, m2):
            m[1].running_mean.copy_(torch.linspace(-0.5, 0.5, cout))
    x = (torch.randn(6, cin, hw, hw) * 1.5 + 0.3).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    assert ewvit.conv.bn_stat_rows(x, m1[0].weight, stride) > 0
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ho = (hw - 1) // stride + 1
    dy = torch.randn(6, cout, ho, ho, device=DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    y2 = m2(x2)                                   # uncapped
    y2.backward(dy)
    with ewvit._lib.grid_cap(cap):
        y1 = m1(x1)
        y1.backward(dy)
    torch.cuda.synchronize()
    assert rel(y1.float(), y2.float()) <= 2 ** -8   # a bf16 step where the batch mean differs in its last bits
    assert rel(m1[1].running_mean, m2[1].running_mean) <= 1e-5
    assert rel(m1[1].running_var, m2[1].running_var) <= 1e-5
    assert rel(x1.grad.float(), x2.grad.float()) <= 2 ** -7
    assert rel(m1[0].weight.grad, m2[0].weight.grad) <= 1e-3
    assert rel(m1[1].weight.grad, m2[1].weight.grad) <= 1e-3


@pytest.mark.parametrize('cap', [16, 160])
def test_capped_mwt_config1_golden(golden, cap):
    """The whole MWT branch (DWT front end, seperate / multiscale / fusion convs, grouped
    BatchNorm) train forward + backward under a cap, against the reference-generated
    fixture (BASELINE configs[0], ref_mwt_cfg1.npz) with the uncapped test's bounds
    (test_gpu_modules.test_mwt_config1_golden).  Capped and uncapped runs differ only in
    the summation order of BatchNorm statistics and weight-gradient splits: bf16 output
    roundings flip, and the small-batch BatchNorm backward amplifies them in the
    gradients, so the two are compared by cosine (conv biases before a train-mode
    BatchNorm have a zero true gradient and are left out)."""
    import ewvit
    from network import mwt
    from oracle.weights import apply_recipe
    from test_gpu_modules import check, cos, log
    z = golden('ref_mwt_cfg1.npz')
    x = torch.from_numpy(z['x']).to(DEV)
    runs = {}
    for c in (0, cap):
        m = apply_recipe(mwt.MWT(3, 64, 2), 11).to(DEV).train()
        with ewvit._lib.grid_cap(c):
            with torch.autocast('cuda', dtype=torch.bfloat16):
                y = m(x)
            (y.float() * torch.from_numpy(z['loss_w']).to(DEV)).sum().backward()
        torch.cuda.synchronize()
        runs[c] = (y.detach(), m)
    y, m = runs[cap]
    check(y, torch.from_numpy(z['y_train']), 2e-2)
    pp = dict(m.named_parameters())
    for k, f in {'hf_conv.fusion.0.weight': 0.98, 'hf_conv.seperate.0.0.weight': 0.98,
                 'freq_pool.1.weight': 0.98}.items():
        c = cos(pp[k].grad, torch.from_numpy(z['grad.' + k]))
        log('grad_cos:' + k, c, f)
        assert c >= f, (k, c, f)
    st = m.state_dict()
    for k in ['hf_conv.fusion.1.running_mean', 'hf_conv.fusion.1.running_var', 'multiscale_fusion.1.running_mean']:
        check(st[k], torch.from_numpy(z['state.' + k]), 2e-2)
    p0 = dict(runs[0][1].named_parameters())
    for k, p in pp.items():
        if k.endswith('.0.bias') or k.endswith('freq_pool.1.bias'):
            continue
        c = cos(p.grad, p0[k].grad)
        log('cap_vs_uncapped_grad_cos:' + k, c, 0.99)
        assert c >= 0.99, (k, c)
