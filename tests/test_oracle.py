"""Pin the oracle (CPU restatement) against the reference-generated fixtures and
pywt.  CPU only — these tests never touch the product package."""
import numpy as np
import pytest
import torch

from oracle import dwt as odwt
from oracle import model as om
from oracle.effnetv2 import EfficientNetV2S
from oracle.weights import apply_recipe, recipe_input

RTOL = 1e-4


def close(a, b, rtol=RTOL, atol=1e-5):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    scale = max(np.abs(b).max(), 1e-6)
    err = np.abs(a - b).max()
    assert err <= atol + rtol * scale, f'max err {err} vs scale {scale}'


def compact_check(actual, z, key, rtol=RTOL):
    a = actual.detach().numpy() if torch.is_tensor(actual) else actual
    if key in z.files:
        close(a, z[key], rtol)
    else:
        close(a.reshape(-1)[:4096], z[key + '@head'], rtol)
        close(a.reshape(a.shape[0], -1).astype(np.float64).sum(1), z[key + '@rowsum'], 1e-3, 1e-3)


def no_stochastic(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        if hasattr(mod, 'sd_prob'):
            mod.sd_prob = 0.0
    return m


def test_dwt_vs_pywt(golden):
    z = golden('dwt_pywt.npz')
    for name, L in (('a', 3), ('b', 3), ('odd', 2)):
        cur = z[f'{name}.x']
        for lv in range(1, L + 1):
            cur, yh = odwt.haar_level(cur)
            np.testing.assert_allclose(cur, z[f'{name}.L{lv}.ll'], atol=1e-6, rtol=1e-6)
            np.testing.assert_allclose(yh, z[f'{name}.L{lv}.yh'], atol=1e-6, rtol=1e-6)


def test_dwt_numpy_equals_torch_afb2d():
    x = recipe_input((2, 3, 32, 32), seed=5)
    ll_t, yh_t = om.DWTForward()(x)
    ll_n, yh_n = odwt.haar_level(x.numpy())
    np.testing.assert_allclose(ll_t.numpy(), ll_n, atol=1e-6)
    np.testing.assert_allclose(yh_t[0].numpy(), yh_n, atol=1e-6)


def test_hf_upsample_matches_torch_interpolate():
    x = recipe_input((2, 3, 64, 48), seed=6)
    up = odwt.hf_upsampled(x.numpy(), 3)
    cur = x
    for lv in range(3):
        ll, yh = om.DWTForward()(cur)
        b, c = cur.shape[:2]
        hf = yh[0].reshape(b, 3 * c, yh[0].shape[-2], yh[0].shape[-1])
        hf = torch.nn.functional.interpolate(hf, size=(32, 24), mode='bilinear')
        np.testing.assert_allclose(up[lv], hf.numpy(), atol=2e-6)
        cur = ll


def test_effnetv2s_param_count():
    m = EfficientNetV2S()
    assert sum(p.numel() for p in m.parameters()) == 21_458_488


def test_mwt_config1(golden):
    z = golden('ref_mwt_cfg1.npz')
    mwt = apply_recipe(om.MWT(3, 64, 2), seed=11)
    x = torch.from_numpy(z['x'])
    mwt.eval()
    with torch.no_grad():
        close(mwt(x), z['y_eval'])
        ll, hf = mwt.wavelet_transform(x, (32, 32))
        close(ll, z['wt_ll'])
        compact_check(hf, z, 'wt_hf')
    mwt.train()
    y = mwt(x)
    close(y, z['y_train'])
    (y * torch.from_numpy(z['loss_w'])).sum().backward()
    sd = dict(mwt.named_parameters())
    for k in ['multiscale_fusion.0.weight', 'hf_conv.seperate.0.0.weight', 'hf_conv.fusion.0.weight',
              'freq_pool.1.weight', 'freq_conv.0.bias']:
        compact_check(sd[k].grad, z, 'grad.' + k, rtol=1e-3)
    st = mwt.state_dict()
    for k in ['hf_conv.fusion.1.running_mean', 'hf_conv.fusion.1.running_var', 'multiscale_fusion.1.running_mean']:
        close(st[k], z['state.' + k])
    assert int(st['hf_conv.fusion.1.num_batches_tracked']) == int(z['state.hf_conv.fusion.1.num_batches_tracked']) == 2


def test_cross_transformer(golden):
    z = golden('ref_cross.npz')
    bct = no_stochastic(apply_recipe(om.BidirectionalCrossTransformer(128, depth=2, heads=4, dim_head=32, dropout=0.1), seed=12))
    s = torch.from_numpy(z['s']).requires_grad_(True)
    f = torch.from_numpy(z['f']).requires_grad_(True)
    so, fo = bct(s, f)
    close(so, z['s_out'])
    close(fo, z['f_out'])
    ((so * torch.from_numpy(z['ws'])).sum() + (fo * torch.from_numpy(z['wf'])).sum()).backward()
    close(s.grad, z['grad.s'], 1e-3)
    close(f.grad, z['grad.f'], 1e-3)
    for n, p in bct.named_parameters():
        close(p.grad, z['grad.' + n], 1e-3)


def test_vit_transformer(golden):
    z = golden('ref_vit.npz')
    cfg = om.ARCH_CONFIG['model']
    tr = no_stochastic(apply_recipe(om.Transformer(cfg['dim'], cfg['depth'], cfg['heads'], cfg['dim-head'], cfg['mlp-dim'], cfg['dropout']), seed=13))
    x = torch.from_numpy(z['x']).requires_grad_(True)
    y = tr(x)
    close(y, z['y'])
    (y * torch.from_numpy(z['w'])).sum().backward()
    close(x.grad, z['grad.x'], 1e-3)
    sd = dict(tr.named_parameters())
    for k in ['layers.0.0.fn.to_qkv.weight', 'layers.1.1.fn.net.0.weight', 'layers.1.1.fn.net.3.bias',
              'layers.0.0.norm.weight', 'layers.1.0.fn.to_out.0.weight']:
        compact_check(sd[k].grad, z, 'grad.' + k, rtol=1e-3)


@pytest.mark.slow
def test_dama_224(golden):
    z = golden('ref_dama.npz')
    torch.manual_seed(0)
    dama = no_stochastic(apply_recipe(om.DAMA(3, 128, 4, 3, batch_size=4), seed=14))
    dama.eval()
    with torch.no_grad():
        feat = recipe_input((4, 1280, 7, 7), seed=1005)
        close(dama.sfe.head(feat), z['head_out'])
        xf = recipe_input((4, 3, 224, 224), seed=1006)
        pf = dama._process_frame(xf)
        for k in ('fused', 'space', 'freq'):
            close(pf[k], z['pf_eval.' + k], 1e-3)
        close(dama.sfe.efficient_net.features(xf).sum(dim=(2, 3)), z['bb_eval_sum'], 1e-3)
        close(dama.mwt(xf), z['mwt_eval'], 1e-3)
    dama.train()
    xv = recipe_input((1, 8, 3, 224, 224), seed=1007)
    res = dama(xv, batch_size=4)
    loss = 0
    for k in res:
        close(res[k], z['fwd.' + k], 1e-3)
        loss = loss + (res[k] * torch.from_numpy(z['lw.' + k])).sum()
    loss.backward()
    sd = dict(dama.named_parameters())
    for k in ['sfe.patch_to_embedding.bias', 'sfe.transformer.layers.1.1.fn.net.3.weight', 'sfe.pos_embedding',
              'sfe.cls_token', 'cross_att.layers.0.1.to_q.weight',
              'mwt.hf_conv.seperate.2.0.weight', 'fusion_gate.0.weight', 'gate_net.5.weight',
              'sfe.efficient_net.features.7.0.weight', 'sfe.efficient_net.features.6.14.block.2.fc1.weight']:
        compact_check(sd[k].grad, z, 'grad.' + k, rtol=2e-3)
    # a conv bias feeding a train-mode BatchNorm has an exactly-zero true gradient:
    # both sides hold only rounding noise, so check magnitude, not value
    g = sd['mwt.multiscale_fusion.0.bias'].grad
    assert g.abs().max() < 1e-3 and np.abs(z['grad.mwt.multiscale_fusion.0.bias']).max() < 1e-3
    close(sd['sfe.patch_to_embedding.weight'].grad.sum(1), z['grad.sfe.patch_to_embedding.weight.rowsum'], 2e-3)
