"""Generate the reference-pinned golden fixtures (tests/golden/ref_*.npz).

Runs the REFERENCE's own ``network/mwt.py``, ``network/sfe.py`` and
``network/dama.py`` from /root/reference (build container only; the reference
never travels) on seeded inputs with the deterministic weight recipe of
``oracle/weights.py`` and stores inputs/outputs/gradients as small .npz files.

Third-party packages the reference imports are absent from the image, so they
are provided as restatements (the same ones the oracle uses):
* ``pytorch_wavelets.DWTForward``      -> oracle.model.DWTForward (pinned by pywt,
                                          see gen_pywt_golden.py)
* ``torchvision.models.efficientnet_v2_s`` -> oracle.effnetv2 (random init; the
                                          IMAGENET1K_V1 weights are unreachable)
* ``efficientnet_pytorch.EfficientNet`` -> an empty placeholder module (only the out-of-scope
                                          b0 ablation heads use it; its weights are a fetch)
* ``cv2``                              -> empty module (imported but unused by sfe.py)

Usage:  python tests/golden/gen_reference_golden.py
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from oracle import effnetv2                      # noqa: E402
from oracle.model import DWTForward as _DWT      # noqa: E402
from oracle.weights import apply_recipe, recipe_input  # noqa: E402


def install_stubs():
    pw = types.ModuleType('pytorch_wavelets')

    class DWTForward(_DWT):
        def __init__(self, J=1, wave='haar', mode='zero'):
            assert (J, wave, mode) == (1, 'haar', 'zero')
            super().__init__()
    pw.DWTForward = DWTForward
    sys.modules['pytorch_wavelets'] = pw

    tv = types.ModuleType('torchvision')
    tvm = types.ModuleType('torchvision.models')

    class EfficientNet_V2_S_Weights:
        IMAGENET1K_V1 = 'IMAGENET1K_V1'
    tvm.efficientnet_v2_s = lambda weights=None, **kw: effnetv2.EfficientNetV2S(**kw)
    tvm.EfficientNet_V2_S_Weights = EfficientNet_V2_S_Weights
    tv.models = tvm
    sys.modules['torchvision'] = tv
    sys.modules['torchvision.models'] = tvm

    ep = types.ModuleType('efficientnet_pytorch')

    class EfficientNet(torch.nn.Module):
        """Parameter-free stand-in: the b0 heads (model.py:38-51) are built but never
        called in 'dynamic' mode; their backbone keys are not part of any fixture."""
        @staticmethod
        def from_pretrained(name):
            return EfficientNet()

        def extract_features(self, img):
            raise RuntimeError('efficientnet_pytorch b0 is out of scope (network fetch)')
    ep.EfficientNet = EfficientNet
    sys.modules['efficientnet_pytorch'] = ep
    sys.modules['cv2'] = types.ModuleType('cv2')


def load_reference():
    install_stubs()
    sys.path.insert(0, REF)
    import network.mwt as rmwt       # noqa: F401
    import network.sfe as rsfe
    import network.dama as rdama
    return rmwt, rsfe, rdama


def reference_losses():
    """orthogonal_loss / combined_loss from the reference's train.py:55-91.  train.py
    itself cannot be imported here (its module level needs the dataset stack: cv2,
    facenet, sklearn's data loaders), so the two function definitions are taken from its
    source text and executed alone."""
    import ast
    src = open(os.path.join(REF, 'train.py')).read()
    tree = ast.parse(src)
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in ('orthogonal_loss', 'combined_loss')]
    ns = {'torch': torch, 'F': torch.nn.functional}
    exec(compile(ast.Module(body=fns, type_ignores=[]), os.path.join(REF, 'train.py'), 'exec'), ns)
    return ns['orthogonal_loss'], ns['combined_loss']


def no_stochastic(module):
    """Dropout p=0 and stochastic depth off, so train-mode passes are deterministic."""
    for m in module.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if hasattr(m, 'sd_prob'):
            m.sd_prob = 0.0
    return module


def grads_of(module, names):
    sd = dict(module.named_parameters())
    return {f'grad.{n}': sd[n].grad.detach().numpy().copy() for n in names}


def loss_weights(shape, seed):
    return torch.from_numpy(np.random.default_rng(seed).standard_normal(shape).astype(np.float32))


BIG = 1 << 16


def compact(d):
    """Arrays above 64K elements are stored as their first 4096 flat elements
    plus their sum over every axis but the first (keeps fixtures small)."""
    out = {}
    for k, v in d.items():
        v = v.detach().numpy() if torch.is_tensor(v) else np.asarray(v)
        if v.size > BIG:
            out[k + '@head'] = v.reshape(-1)[:4096].copy()
            out[k + '@rowsum'] = v.reshape(v.shape[0], -1).astype(np.float64).sum(1).astype(np.float32)
        else:
            out[k] = v
    return out


def save(name, d):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **compact(d))
    print('wrote', path, f'{os.path.getsize(path) / 1e6:.2f} MB')


def main():
    torch.manual_seed(0)
    cwd = os.getcwd()
    os.chdir(REF)        # dama.py:94 / model.py:31 read config/architecture.yaml relatively
    try:
        rmwt, rsfe, rdama = load_reference()
        import yaml
        cfg = yaml.safe_load(open('config/architecture.yaml'))

        # ---- G2: MWT config 1 (BASELINE configs[0]): [4,3,64,64], dim 64, 2 levels
        mwt = apply_recipe(rmwt.MWT(in_channels=3, dama_dim=64, levels=2), seed=11)
        x = recipe_input((4, 3, 64, 64), seed=1001)
        mwt.eval()
        with torch.no_grad():
            y_eval = mwt(x)
            ll1, hfc1 = mwt.wavelet_transform(x, (32, 32))
        mwt.train()
        xg = x.clone()
        y_tr = mwt(xg)
        w = loss_weights(tuple(y_tr.shape), 7)
        (y_tr * w).sum().backward()
        out = {'x': x, 'y_eval': y_eval, 'wt_ll': ll1, 'wt_hf': hfc1, 'y_train': y_tr, 'loss_w': w}
        out.update(grads_of(mwt, ['multiscale_fusion.0.weight', 'hf_conv.seperate.0.0.weight',
                                  'hf_conv.fusion.0.weight', 'freq_pool.1.weight', 'freq_conv.0.bias']))
        sd = mwt.state_dict()
        for k in ['hf_conv.fusion.1.running_mean', 'hf_conv.fusion.1.running_var',
                  'multiscale_fusion.1.running_mean', 'hf_conv.fusion.1.num_batches_tracked']:
            out['state.' + k] = sd[k]
        save('ref_mwt_cfg1.npz', out)

        # ---- G3: BidirectionalCrossTransformer dim 128, heads 4, depth 2 (dama.py:116-122)
        bct = no_stochastic(apply_recipe(rdama.BidirectionalCrossTransformer(128, depth=2, heads=4, dim_head=32, dropout=0.1), seed=12))
        bct.train()
        s = recipe_input((16, 1, 128), seed=1002).requires_grad_(True)
        f = recipe_input((16, 1, 128), seed=1003).requires_grad_(True)
        so, fo = bct(s, f)
        ws, wf = loss_weights(tuple(so.shape), 8), loss_weights(tuple(fo.shape), 9)
        ((so * ws).sum() + (fo * wf).sum()).backward()
        out = {'s': s.detach(), 'f': f.detach(), 's_out': so, 'f_out': fo, 'ws': ws, 'wf': wf,
               'grad.s': s.grad, 'grad.f': f.grad}
        out.update(grads_of(bct, [n for n, _ in bct.named_parameters()]))
        save('ref_cross.npz', out)

        # ---- G4: ViT Transformer, full size (sfe.py:72-85 with architecture.yaml dims)
        m = cfg['model']
        tr = no_stochastic(apply_recipe(rsfe.Transformer(m['dim'], m['depth'], m['heads'], m['dim-head'], m['mlp-dim'], m['dropout']), seed=13))
        tr.train()
        xt = recipe_input((16, 2, 512), seed=1004).requires_grad_(True)
        yt = tr(xt)
        wt = loss_weights(tuple(yt.shape), 10)
        (yt * wt).sum().backward()
        out = {'x': xt.detach(), 'y': yt, 'w': wt, 'grad.x': xt.grad}
        out.update(grads_of(tr, ['layers.0.0.fn.to_qkv.weight', 'layers.1.1.fn.net.0.weight',
                                 'layers.1.1.fn.net.3.bias', 'layers.0.0.norm.weight', 'layers.1.0.fn.to_out.0.weight']))
        save('ref_vit.npz', out)

        # ---- G5 + G6: DAMA at 224 (dama.py:130-206) with recipe weights.
        dama = no_stochastic(apply_recipe(rdama.DAMA(in_channels=3, dim=128, num_heads=4, levels=3, batch_size=4), seed=14))
        # G5: EfficientViT head on a fixed backbone map (sfe.py:153-173)
        feat = recipe_input((4, 1280, 7, 7), seed=1005)
        dama.eval()
        with torch.no_grad():
            head_out = rsfe_head(dama.sfe, feat)
            xf = recipe_input((4, 3, 224, 224), seed=1006)
            pf_eval = dama._process_frame(xf)
            bb_eval = dama.sfe.efficient_net.features(xf)
            mwt_eval = dama.mwt(xf)
        out = {'feat': feat, 'head_out': head_out, 'pf_eval.fused': pf_eval['fused'],
               'pf_eval.space': pf_eval['space'], 'pf_eval.freq': pf_eval['freq'],
               'bb_eval_sum': bb_eval.sum(dim=(2, 3)), 'mwt_eval': mwt_eval}
        # G6: train mode (BN batch stats), forward over K=8 frames in 2 chunks of 4 + backward
        dama.train()
        xv = recipe_input((1, 8, 3, 224, 224), seed=1007)
        res = dama(xv, batch_size=4)
        wl = {k: loss_weights(tuple(v.shape), 20 + i) for i, (k, v) in enumerate(sorted(res.items()))}
        sum((res[k] * wl[k]).sum() for k in res).backward()
        for k in res:
            out[f'fwd.{k}'] = res[k]
            out[f'lw.{k}'] = wl[k]
        out.update(grads_of(dama, ['sfe.patch_to_embedding.bias', 'sfe.transformer.layers.1.1.fn.net.3.weight',
                                   'sfe.pos_embedding', 'sfe.cls_token', 'cross_att.layers.0.1.to_q.weight',
                                   'mwt.multiscale_fusion.0.bias', 'mwt.hf_conv.seperate.2.0.weight',
                                   'fusion_gate.0.weight', 'gate_net.5.weight',
                                   'sfe.efficient_net.features.7.0.weight',
                                   'sfe.efficient_net.features.6.14.block.2.fc1.weight']))
        out['grad.sfe.patch_to_embedding.weight.rowsum'] = dama.sfe.patch_to_embedding.weight.grad.sum(1)
        save('ref_dama.npz', out)

        # ---- G7: DeepfakeDetector 'dynamic' (model.py:70-99): logits in eval and train mode,
        # classifier gradients, and the reference state-dict key/shape manifest
        import network.model as rmodel
        det = no_stochastic(apply_recipe(rmodel.DeepfakeDetector(3, 128, batch_size=4), seed=15))
        xd = recipe_input((2, 4, 3, 224, 224), seed=1008)
        det.eval()
        with torch.no_grad():
            ev = det(xd, 4, 'dynamic')
        det.train()
        tr = det(xd, 4, 'dynamic')
        wlog = loss_weights(tuple(tr['logits'].shape), 30)
        (tr['logits'] * wlog).sum().backward()
        out = {'x': xd, 'eval.logits': ev['logits'], 'eval.fused': ev['fused'], 'train.logits': tr['logits'],
               'train.fused': tr['fused'], 'train.space': tr['space'], 'train.freq': tr['freq'], 'lw': wlog}
        out.update(grads_of(det, ['classifier.0.weight', 'classifier.0.bias', 'classifier.3.weight',
                                  'classifier.3.bias', 'dama.gate_net.5.weight']))
        sd = det.state_dict()
        keys = list(sd.keys())
        out['manifest.keys'] = np.array(keys)
        out['manifest.shapes'] = np.array([list(sd[k].shape) + [-1] * (4 - sd[k].dim()) for k in keys], dtype=np.int64)
        save('ref_detector.npz', out)

        # ---- G8: combined_loss / orthogonal_loss (train.py:55-91) at three curriculum points
        r_orth, r_comb = reference_losses()
        crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5]))
        out = {}
        logits0 = recipe_input((8, 1), seed=1009)
        space0 = recipe_input((8, 128), seed=1010)
        freq0 = recipe_input((8, 128), seed=1011) + 0.3 * space0
        labels = torch.tensor([1., 0., 1., 1., 0., 0., 1., 0.])
        out.update({'logits': logits0, 'space': space0, 'freq': freq0, 'labels': labels,
                    'orth': r_orth(space0, freq0)})
        for epoch, maxe in ((1, 10), (4, 10), (9, 10)):
            lg, sp, fq = (t.clone().requires_grad_(True) for t in (logits0, space0, freq0))
            loss, _ = r_comb({'logits': lg, 'space': sp, 'freq': fq}, labels, crit, epoch, maxe)
            loss.backward()
            tag = f'e{epoch}of{maxe}'
            out[f'{tag}.loss'] = loss.detach()
            out[f'{tag}.grad.logits'] = lg.grad
            out[f'{tag}.grad.space'] = sp.grad if sp.grad is not None else torch.zeros_like(sp)
            out[f'{tag}.grad.freq'] = fq.grad if fq.grad is not None else torch.zeros_like(fq)
        save('ref_loss.npz', out)
    finally:
        os.chdir(cwd)


def rsfe_head(sfe, feat):
    """Run the reference EfficientViT.forward (sfe.py:145-173) with the backbone
    replaced by identity so `feat` is the [B,1280,7,7] map."""
    saved = sfe.efficient_net.features
    sfe.efficient_net.features = torch.nn.Identity()
    try:
        return sfe(feat)
    finally:
        sfe.efficient_net.features = saved


if __name__ == '__main__':
    main()
