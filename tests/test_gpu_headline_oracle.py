"""The headline shape against the oracle.

BASELINE config 2 is ONE 64-frame `_process_frame` chunk: x = [8, 8, 3, 224, 224] with
batch_size=8 (reference dama.py:179-186), so every train-mode BatchNorm normalises over 64
frames and `pos_embedding[0:64]` is indexed by the frame's chunk position (sfe.py:126,158-159).
The product's eager train step at exactly that shape — DeepfakeDetector (model.py:70-99),
combined_loss with the orthogonality term on (train.py:69-91, epoch 1 of 1), bf16 — is
compared with the fp32 CPU oracle on the same recipe weights and inputs, dropout and
stochastic depth off:

* outputs `fused` / `space` / `freq` / `logits` and the loss (max |err| <= 2e-2 of
  scale, cosine >= 0.999);
* every `pos_embedding` row 0..63 gets its gradient from its own frames only: per-row cosine;
* a set of weight gradients across the MWT, the backbone, the ViT, the cross-attention, the
  gates and the classifier;
* the BatchNorm running statistics after the step.

The oracle at 64 frames runs fwd + bwd in ~10-20 s on the box's host cores.
"""
import copy
import os

import pytest
import torch

from test_gpu_modules import check, cos, log, no_stochastic

pytestmark = pytest.mark.gpu
DEV = 'cuda'

OUT_TOL, OUT_COS = 2e-2, 0.999
POS_ROW_COS = 0.99                      # each pos_embedding row (one frame position of 8 videos)
GRAD_COS = {
    'classifier.3.weight': 0.999,
    'classifier.0.weight': 0.995,
    'dama.gate_net.2.weight': 0.99,
    'dama.gate_net.5.weight': 0.99,
    'dama.fusion_gate.0.weight': 0.99,
    'dama.cross_att.layers.0.1.to_q.weight': 0.99,
    'dama.cross_att.layers.1.3.to_kv.weight': 0.99,
    'dama.cross_att.layers.0.0.weight': 0.99,
    'dama.sfe.feat_map.0.weight': 0.99,
    'dama.sfe.transformer.layers.0.0.fn.to_qkv.weight': 0.99,
    'dama.sfe.transformer.layers.1.1.fn.net.0.weight': 0.99,
    'dama.sfe.patch_to_embedding.weight': 0.99,
    'dama.sfe.cls_token': 0.99,
    'dama.sfe.efficient_net.features.7.0.weight': 0.98,
    'dama.sfe.efficient_net.features.6.3.block.1.0.weight': 0.97,
    'dama.sfe.efficient_net.features.2.1.block.0.0.weight': 0.95,
    'dama.mwt.multiscale_fusion.0.weight': 0.99,
    'dama.mwt.hf_conv.fusion.0.weight': 0.99,
    'dama.mwt.hf_conv.seperate.1.0.weight': 0.99,
    'dama.mwt.freq_conv.0.weight': 0.99,
    'dama.mwt.freq_pool.1.weight': 0.99,
}
STAT_TOL = 2e-2
STATS = ['dama.mwt.hf_conv.fusion.1.running_mean', 'dama.mwt.hf_conv.seperate.2.1.running_var',
         'dama.mwt.multiscale_fusion.1.running_var', 'dama.mwt.freq_pool.2.running_mean',
         'dama.fusion_gate.1.running_mean', 'dama.fusion_gate.1.running_var',
         'dama.sfe.efficient_net.features.7.1.running_var', 'dama.sfe.efficient_net.features.4.2.block.1.1.running_mean']


def test_headline_chunk_train_step_vs_oracle():
    from network.losses import combined_loss
    from network.model import DeepfakeDetector
    from oracle import model as om
    from oracle.weights import recipe_input, recipe_state_dict
    torch.set_num_threads(max(1, min(32, len(os.sched_getaffinity(0)))))
    o = no_stochastic(om.DeepfakeDetector(3, 128, batch_size=8))
    p = DeepfakeDetector(3, 128, batch_size=8)
    sd = recipe_state_dict(p.state_dict(), 15)
    p.load_state_dict(sd)
    o.load_state_dict({k: v for k, v in sd.items() if k in o.state_dict()})
    p = no_stochastic(p).to(DEV).to(memory_format=torch.channels_last).train()
    o.train()
    x = recipe_input((8, 8, 3, 224, 224), seed=2024)
    labels = torch.tensor([0., 1., 1., 0., 1., 0., 0., 1.])
    pw = torch.tensor([0.5])

    ro = o(x, 8, 'dynamic')
    lo = om.combined_loss(ro, labels, torch.nn.BCEWithLogitsLoss(pos_weight=pw), 1, 1)
    lo.backward()

    with torch.autocast('cuda', dtype=torch.bfloat16):
        rp = p(x.to(DEV), 8, 'dynamic')
    lp, _ = combined_loss(rp, labels.to(DEV), torch.nn.BCEWithLogitsLoss(pos_weight=pw.to(DEV)), 1, 1)
    lp.backward()
    torch.cuda.synchronize()

    for k in ('fused', 'space', 'freq', 'logits'):
        check(rp[k], ro[k], OUT_TOL, OUT_COS)
    el = abs(float(lp) - float(lo)) / abs(float(lo))
    log('loss_rel', el, OUT_TOL)
    assert el <= OUT_TOL, (float(lp), float(lo))

    pp, oo = dict(p.named_parameters()), dict(o.named_parameters())
    # pos_embedding: row n is frame position n of the 64-frame chunk (sfe.py:158-159)
    gp, go = pp['dama.sfe.pos_embedding'].grad, oo['dama.sfe.pos_embedding'].grad
    assert gp.shape[0] == 64
    rows = [cos(gp[n], go[n]) for n in range(64)]
    log('pos_row_cos_min', min(rows), POS_ROW_COS)
    assert min(rows) >= POS_ROW_COS, [(n, c) for n, c in enumerate(rows) if c < POS_ROW_COS]
    assert bool((gp.reshape(64, -1).abs().amax(1) > 0).all())
    fails = []
    for n, f in GRAD_COS.items():
        assert pp[n].grad is not None and oo[n].grad is not None, n
        c = cos(pp[n].grad, oo[n].grad)
        nr = float(pp[n].grad.norm()) / max(float(oo[n].grad.norm()), 1e-30)
        log('grad_cos:' + n, c, f)
        log('grad_norm_ratio:' + n, nr, 0.05)
        if c < f or abs(nr - 1) > 0.05:
            fails.append((n, round(c, 5), round(nr, 4)))
    assert not fails, fails
    ps, os_ = p.state_dict(), o.state_dict()
    for k in STATS:
        check(ps[k], os_[k], STAT_TOL, 0.999)
    for k in ('dama.mwt.hf_conv.fusion.1.num_batches_tracked', 'dama.fusion_gate.1.num_batches_tracked'):
        assert int(ps[k]) == int(os_[k]), k
