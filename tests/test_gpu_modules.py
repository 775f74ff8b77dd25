"""Module-level parity: the product (efficient-wavelet-vit_amd/network on ewvit
kernels, MI355X) against the oracle (CPU fp32 restatement pinned to the
reference) with identical recipe weights and inputs.

Tolerance: bf16 GPU vs fp32 CPU — max |err| <= 2e-2 * scale of the
output and cosine >= 0.999 for modules and eval-mode passes; gradients cosine >= 0.99
(bf16 operands in every GEMM/conv).  The full DAMA / detector TRAIN step (train-mode
BatchNorm over 8-frame chunks, ~300 layers) has its own fixed bounds, justified next to
TRAIN_OUT_TOL below.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def cos(a, b):
    a = a.detach().double().flatten().cpu()
    b = b.detach().double().flatten().cpu()
    return float((a @ b) / (a.norm() * b.norm() + 1e-30))


_LOG = os.environ.get('EWVIT_PARITY_LOG')


def log(kind, value, bound):
    """EWVIT_PARITY_LOG=path: every measured error / cosine next to its bound (JSON lines)."""
    if _LOG:
        with open(_LOG, 'a') as f:
            f.write(json.dumps({'test': os.environ.get('PYTEST_CURRENT_TEST', '').split(' ')[0], 'kind': kind,
                                'value': value, 'bound': bound}) + '\n')


def check(a, b, tol=2e-2, cmin=0.999):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    scale = max(float(b.abs().max()), 1e-6)
    err = float((a - b).abs().max())
    c = cos(a, b)
    log('err_of_scale', err / scale, tol)
    log('cos', c, cmin)
    assert err <= tol * scale and c >= cmin, f'max err {err:.3e} (scale {scale:.3e}), cos {c:.6f}'


def no_stochastic(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        if hasattr(mod, 'sd_prob'):
            mod.sd_prob = 0.0
    return m


def pair(prod_cls, oracle_cls, args, seed):
    from oracle.weights import recipe_state_dict
    o = no_stochastic(oracle_cls(*args))
    sd = recipe_state_dict(o.state_dict(), seed)
    o.load_state_dict(sd)
    p = no_stochastic(prod_cls(*args))
    p.load_state_dict(sd)
    return p.to(DEV), o


def grads_close(p, o, names, cmin=0.99):
    pp, oo = dict(p.named_parameters()), dict(o.named_parameters())
    for n in names:
        assert pp[n].grad is not None, n
        c = cos(pp[n].grad, oo[n].grad)
        assert c >= cmin, f'{n}: grad cosine {c:.5f}'


def test_vit_transformer_vs_oracle():
    from network import sfe
    from oracle import model as om
    from oracle.weights import recipe_input
    p, o = pair(sfe.Transformer, om.Transformer, (512, 2, 8, 64, 2048, 0.15), 13)
    p.train(); o.train()
    x = recipe_input((64, 2, 512), 77)
    xo = x.clone().requires_grad_(True)
    xp = x.to(DEV).requires_grad_(True)
    yo, yp = o(xo), p(xp)
    check(yp, yo)
    w = torch.randn(yo.shape, generator=torch.Generator().manual_seed(1))
    (yo * w).sum().backward()
    (yp * w.to(DEV)).sum().backward()
    assert cos(xp.grad, xo.grad) > 0.995
    grads_close(p, o, [n for n, _ in o.named_parameters()])


def test_vit_golden(golden):
    """Straight against the reference-generated fixture (ref_vit.npz)."""
    from network import sfe
    from oracle.weights import apply_recipe
    z = golden('ref_vit.npz')
    tr = no_stochastic(apply_recipe(sfe.Transformer(512, 2, 8, 64, 2048, 0.15), 13)).to(DEV)
    x = torch.from_numpy(z['x']).to(DEV).requires_grad_(True)
    y = tr(x)
    check(y, torch.from_numpy(z['y']))
    (y * torch.from_numpy(z['w']).to(DEV)).sum().backward()
    check(x.grad, torch.from_numpy(z['grad.x']), tol=3e-2, cmin=0.995)


def test_cross_transformer_vs_golden(golden):
    from network import dama
    from oracle.weights import apply_recipe
    z = golden('ref_cross.npz')
    bct = no_stochastic(apply_recipe(dama.BidirectionalCrossTransformer(128, 2, 4, 32, 0.1), 12)).to(DEV)
    s = torch.from_numpy(z['s']).to(DEV).requires_grad_(True)
    f = torch.from_numpy(z['f']).to(DEV).requires_grad_(True)
    so, fo = bct(s, f)
    check(so, torch.from_numpy(z['s_out']))
    check(fo, torch.from_numpy(z['f_out']))
    ((so * torch.from_numpy(z['ws']).to(DEV)).sum() + (fo * torch.from_numpy(z['wf']).to(DEV)).sum()).backward()
    check(s.grad, torch.from_numpy(z['grad.s']), tol=3e-2, cmin=0.995)
    check(f.grad, torch.from_numpy(z['grad.f']), tol=3e-2, cmin=0.995)
    for n, prm in bct.named_parameters():
        assert cos(prm.grad, torch.from_numpy(z['grad.' + n])) > 0.99, n


@pytest.mark.parametrize('autocast', [False, True])
def test_mwt_config1_golden(golden, autocast):
    """BASELINE configs[0]: MWT(3, 64, levels=2) on [4,3,64,64], eval and train."""
    from network import mwt
    from oracle.weights import apply_recipe
    z = golden('ref_mwt_cfg1.npz')
    m = apply_recipe(mwt.MWT(3, 64, 2), 11).to(DEV)
    x = torch.from_numpy(z['x']).to(DEV)
    tol = 2e-2
    m.eval()
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, enabled=autocast):
        check(m(x), torch.from_numpy(z['y_eval']), tol)
    m.train()
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=autocast):
        y = m(x)
    check(y, torch.from_numpy(z['y_train']), tol)
    (y.float() * torch.from_numpy(z['loss_w']).to(DEV)).sum().backward()
    # fixed gradient bound: the MWT conv kernels take bf16 operands with or without autocast
    floor = {'hf_conv.fusion.0.weight': 0.98, 'hf_conv.seperate.0.0.weight': 0.98,
             'freq_pool.1.weight': 0.98}
    pp = dict(m.named_parameters())
    for k, f in floor.items():
        c = cos(pp[k].grad, torch.from_numpy(z['grad.' + k]))
        log('grad_cos:' + k, c, f)
        assert c >= f, (k, c, f)
    st = m.state_dict()
    for k in ['hf_conv.fusion.1.running_mean', 'hf_conv.fusion.1.running_var', 'multiscale_fusion.1.running_mean']:
        check(st[k], torch.from_numpy(z['state.' + k]), tol)
    assert int(st['hf_conv.fusion.1.num_batches_tracked']) == 2
    assert int(st['hf_conv.seperate.1.1.num_batches_tracked']) == 2


def test_mwt_wavelet_transform_api_and_patched_path(golden):
    """The per-level API (mwt.py:74-90) and the monkey-patch fallback
    (utils/visualize_feature_maps.py:151-158) give the fast path's result."""
    from network import mwt
    from oracle.weights import apply_recipe
    z = golden('ref_mwt_cfg1.npz')
    m = apply_recipe(mwt.MWT(3, 64, 2), 11).to(DEV).eval()
    x = torch.from_numpy(z['x']).to(DEV)
    with torch.no_grad():
        ll, hf = m.wavelet_transform(x, (32, 32))
        check(ll, torch.from_numpy(z['wt_ll']), 1e-5)
        fast = m(x)
        orig = m.wavelet_transform
        calls = []

        def spy(xx, ts):
            calls.append(xx.shape)
            return orig(xx, ts)
        m.wavelet_transform = spy
        slow = m(x)
    assert len(calls) == 2
    check(slow, fast, 2e-2)  # per-level path: library convs in fp32 vs the bf16 MFMA path


def test_dwt_module_api():
    from network.mwt import DWTForward
    from oracle.model import DWTForward as ODWT
    x = torch.randn(2, 3, 32, 32)
    ll, yh = DWTForward().to(DEV)(x.to(DEV))
    llo, yho = ODWT()(x)
    torch.testing.assert_close(ll.cpu(), llo, atol=1e-6, rtol=0)
    torch.testing.assert_close(yh[0].cpu(), yho[0], atol=1e-6, rtol=0)
    assert set(DWTForward().state_dict()) == {'h0_col', 'h1_col', 'h0_row', 'h1_row'}


@pytest.fixture(scope='module')
def dama_pair():
    from network import dama
    from oracle import model as om
    torch.manual_seed(0)
    return pair(dama.DAMA, om.DAMA, (3, 128, 4, 3, 8), 14)


def test_efficientvit_head_golden(golden, dama_pair):
    p, _ = dama_pair
    z = golden('ref_dama.npz')
    from oracle.weights import recipe_input
    feat = recipe_input((4, 1280, 7, 7), seed=1005).to(DEV).to(memory_format=torch.channels_last)
    p.eval()
    with torch.no_grad():
        check(p.sfe.head(feat), torch.from_numpy(z['head_out']))


def test_dama_process_frame_eval_golden(golden, dama_pair):
    p, _ = dama_pair
    z = golden('ref_dama.npz')
    from oracle.weights import recipe_input
    xf = recipe_input((4, 3, 224, 224), seed=1006).to(DEV)
    p.eval()
    with torch.no_grad():
        out = p._process_frame(xf)
        for k in ('fused', 'space', 'freq'):
            check(out[k], torch.from_numpy(z['pf_eval.' + k]))
        check(p.mwt(xf), torch.from_numpy(z['mwt_eval']))


def _max_err(a, b):
    return float((a.detach().float().cpu() - b.detach().float().cpu()).abs().max())


# Fixed parity bounds of the full DAMA train step (bf16 MFMA operands, BatchNorm batch
# statistics over 8-frame chunks).  Output bounds from tools/diag_tol.py
# (profiles/r02/diag_tol.json): on these inputs torch's OWN bf16 autocast of the reference op
# sequence reaches max err 0.054 of scale / cosine 0.9989 on `fused`, while torch fp32 on the
# GPU matches the CPU oracle to 1.0 — so the spread is bf16 arithmetic through ~300 layers
# with small-batch BatchNorm, not a kernel defect; the product measures 0.035 / 0.99941
# (DAMA) and up to 0.041 / 0.9992 (DeepfakeDetector, one 8-frame chunk).
TRAIN_OUT_TOL, TRAIN_OUT_COS = 5e-2, 0.999
# Gradient floors from a DISTRIBUTION, not one draw (tools/diag_seeds.py,
# profiles/r02/diag_seeds.json): the gradient cosines of torch's bf16 autocast against the
# fp32 oracle over 4 input seeds (4242, 1, 2, 3); each floor is that minimum minus 0.005
# (rounded down to 0.005) — the product must stay as close to fp32 as torch's own bf16 run
# is in its worst draw.  Layers behind small-batch BatchNorm swing with any change of bf16
# rounding upstream (fusion_gate: a conv on the 1x1 map, then train-mode BN over 8 frames,
# whose backward removes the batch mean and the x_hat projection of dy and scales by 1/sigma
# of 8 samples: autocast 0.928-0.963, product 0.946-0.977 over the seeds).  Product on seed
# 4242 / over the 4 seeds in the comment of each line.
GRAD_FLOOR = {
    'sfe.patch_to_embedding.weight': 0.960,                 # 0.977 / 0.977-0.987
    'sfe.transformer.layers.0.0.fn.to_qkv.weight': 0.975,   # 0.985 / 0.985-0.993
    'sfe.transformer.layers.1.1.fn.net.0.weight': 0.970,    # 0.984 / 0.984-0.992
    'cross_att.layers.1.3.to_kv.weight': 0.990,             # 0.998 / 0.998-0.999
    'cross_att.layers.0.0.weight': 0.985,                   # 0.994 / 0.994-0.997
    'gate_net.2.weight': 0.965,                             # 0.982 / 0.982-0.995
    'sfe.pos_embedding': 0.975,                             # 0.986 / 0.985-0.993
    'sfe.cls_token': 0.985,                                 # 0.993 / 0.993-0.997
    'fusion_gate.0.weight': 0.920,                          # 0.946 / 0.946-0.977
    'mwt.multiscale_fusion.0.weight': 0.965,                # 0.978 / 0.978-0.981
    'mwt.hf_conv.fusion.0.weight': 0.960,                   # 0.976 / 0.976-0.980
    'mwt.hf_conv.seperate.1.0.weight': 0.955,               # 0.974 / 0.973-0.979
    'sfe.efficient_net.features.7.0.weight': 0.945,         # 0.968 / 0.968-0.981
    'sfe.efficient_net.features.6.3.block.1.0.weight': 0.930,   # 0.956 / 0.955-0.970
}
# aggregate over all 326 non-bias weight gradients, same rule: autocast mean 0.942-0.950 /
# min 0.827-0.899 over the seeds; product mean 0.958-0.972, min 0.902-0.942.
# Biases are left out of the aggregate: a per-channel constant that reaches a train-mode
# BatchNorm through linear ops (every conv bias before its BN, the MBConv project-BN biases
# whose residual stream ends in BNs) has an exactly zero true gradient, so its computed
# gradient is rounding noise (cosine -0.5 .. 0.2 even for torch fp32 on the GPU).
GRAD_MEAN_FLOOR, GRAD_MIN_FLOOR = 0.935, 0.82


def test_dama_train_step_vs_oracle(dama_pair):
    """Train-mode DAMA.forward over K=8 frames per video in 2 chunks + backward under bf16
    autocast (the bench's arithmetic), vs the fp32 oracle on CPU (same weights; dropout /
    stochastic depth off), with the fixed bounds above."""
    import copy
    p0, o0 = dama_pair
    p, o = copy.deepcopy(p0), copy.deepcopy(o0)
    p.train(); o.train()
    from oracle.weights import recipe_input
    x = recipe_input((2, 8, 3, 224, 224), seed=4242)
    ro = o(x, batch_size=4)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        rp = p(x.to(DEV), batch_size=4)
    for k in ro:
        check(rp[k], ro[k], TRAIN_OUT_TOL, TRAIN_OUT_COS)
    w = {k: torch.randn(v.shape, generator=torch.Generator().manual_seed(i)) for i, (k, v) in enumerate(sorted(ro.items()))}
    sum((ro[k] * w[k]).sum() for k in ro).backward()
    sum((rp[k].float() * w[k].to(DEV)).sum() for k in rp).backward()
    pp, oo = dict(p.named_parameters()), dict(o.named_parameters())
    for n, f in GRAD_FLOOR.items():
        assert pp[n].grad is not None, n
        c = cos(pp[n].grad, oo[n].grad)
        log('grad_cos:' + n, c, f)
        assert c >= f, f'{n}: grad cosine {c:.5f} < {f}'
    cs = {n: cos(pp[n].grad, g.grad) for n, g in oo.items() if g.grad is not None and not n.endswith('.bias')}
    assert all(pp[n].grad is not None for n in cs)
    mean = sum(cs.values()) / len(cs)
    worst = min(cs.items(), key=lambda kv: kv[1])
    log('grad_cos_mean', mean, GRAD_MEAN_FLOOR)
    log('grad_cos_min:' + worst[0], worst[1], GRAD_MIN_FLOOR)
    assert mean >= GRAD_MEAN_FLOOR and worst[1] >= GRAD_MIN_FLOOR, (mean, worst, len(cs))
    # BatchNorm running statistics were updated per level and per chunk like the reference
    ps, os_ = p.state_dict(), o.state_dict()
    for k in ['mwt.hf_conv.fusion.1.running_mean', 'mwt.hf_conv.seperate.2.1.running_var',
              'fusion_gate.1.running_mean', 'mwt.multiscale_fusion.1.running_var']:
        check(ps[k], os_[k], TRAIN_OUT_TOL)
    assert int(ps['mwt.hf_conv.fusion.1.num_batches_tracked']) == int(os_['mwt.hf_conv.fusion.1.num_batches_tracked']) == 6


def test_chunk_over_64_frames_raises_like_reference(dama_pair):
    p, _ = dama_pair
    with pytest.raises(RuntimeError, match='pos_embedding'):
        p.sfe.head(torch.randn(65, 1280, 7, 7, device=DEV))


@pytest.fixture(scope='module')
def detector_golden():
    """The product DeepfakeDetector with the recipe weights of ref_detector.npz (seed 15;
    the recipe is keyed by state-dict name, and the product's keys are the reference's)."""
    from network.model import DeepfakeDetector
    from oracle.weights import recipe_state_dict
    m = DeepfakeDetector(3, 128, batch_size=4)
    m.load_state_dict(recipe_state_dict(m.state_dict(), 15))
    return no_stochastic(m).to(DEV).to(memory_format=torch.channels_last)


def test_deepfake_detector_eval_vs_reference_golden(golden, detector_golden):
    """A13: DeepfakeDetector.forward(x, batch_size, 'dynamic') (model.py:70-99) in eval mode,
    against the reference's own output (ref_detector.npz, 2 videos x 4 frames, one chunk)."""
    from oracle.weights import recipe_input
    z = golden('ref_detector.npz')
    m = detector_golden.eval()
    x = recipe_input((2, 4, 3, 224, 224), seed=1008).to(DEV)
    with torch.no_grad():
        out = m(x, 4, 'dynamic')
    check(out['fused'], torch.from_numpy(z['eval.fused']))
    check(out['logits'], torch.from_numpy(z['eval.logits']))


DET_GRAD_COS = 0.97      # the train-step gradient floor class of GRAD_FLOOR's token path
# The detector's train step runs ONE 8-frame chunk (2 videos x 4 frames): every train-mode
# BatchNorm sees 8 samples, so its outputs carry more bf16 spread than DAMA's two chunks.
# Fixed from a distribution (tools/diag_detector.py, profiles/r02/diag_detector.json, input
# seeds 1008 1 2 3): torch's own bf16 autocast of the oracle reaches fused 0.035-0.061, space
# 0.036-0.060, freq 0.028-0.052 of scale; the product 0.034-0.054 / 0.028-0.041 / 0.033-0.037
# (seed 1008: fused 0.054).  Bound: autocast's maximum rounded up.
DET_TRAIN_OUT_TOL = 0.065


def test_deepfake_detector_train_vs_reference_golden(golden, detector_golden):
    """A13 in train mode (BatchNorm batch statistics, dropout p=0) + classifier gradients."""
    import copy
    from oracle.weights import recipe_input
    z = golden('ref_detector.npz')
    m = copy.deepcopy(detector_golden).train()
    x = recipe_input((2, 4, 3, 224, 224), seed=1008).to(DEV)
    assert np.allclose(x.reshape(-1)[:4096].cpu().numpy(), z['x@head'])
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = m(x, 4, 'dynamic')
    for k in ('fused', 'space', 'freq', 'logits'):
        check(out[k], torch.from_numpy(z['train.' + k]), DET_TRAIN_OUT_TOL, TRAIN_OUT_COS)
    (out['logits'].float() * torch.from_numpy(z['lw']).to(DEV)).sum().backward()
    pp = dict(m.named_parameters())
    fails = []
    for n in ('classifier.0.weight', 'classifier.0.bias', 'classifier.3.weight', 'classifier.3.bias',
              'dama.gate_net.5.weight'):
        c = cos(pp[n].grad, torch.from_numpy(z['grad.' + n]))
        log('grad_cos:' + n, c, DET_GRAD_COS)
        if c < DET_GRAD_COS:
            fails.append((n, c))
    assert not fails, fails


def test_deepfake_detector_forward_backward_runs():
    from network.model import DeepfakeDetector
    from network.losses import combined_loss
    m = DeepfakeDetector(3, 128, 8).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(2, 8, 3, 224, 224, device=DEV)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = m(x, 8, 'dynamic')
    loss, parts = combined_loss(out, torch.tensor([0., 1.], device=DEV),
                                torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5], device=DEV)), 1, 1)
    loss.backward()
    assert torch.isfinite(loss)
    assert out['logits'].shape == (2, 1)
    assert m.dama.sfe.patch_to_embedding.weight.grad is not None
    assert m.dama.sfe.efficient_net.features[0][0].weight.grad is None      # frozen (sfe.py:115-119)
