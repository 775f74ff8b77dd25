"""Drop-in checks that need no GPU:

* reference checkpoints load into the product's DeepfakeDetector the way the reference's
  eval.py:60-77 loads them — torch.load + strict load_state_dict — including the
  DataParallel ``module.`` prefix (train.py:309,315) and the b0 ablation heads' keys
  (model.py:37-51), and round-trip through state_dict();
* combined_loss / orthogonal_loss (product network/losses.py and the oracle) against the
  values and gradients the reference's own train.py:55-91 produced (ref_loss.npz) at three
  curriculum points, including the device-weight form the replayed step uses.

The reference state-dict manifest (names and shapes of the reference DeepfakeDetector,
1023 keys) comes from ref_detector.npz; the b0 backbone keys, which need efficientnet_pytorch
(absent), are synthesised in its module naming (``_conv_stem``, ``_blocks.N._bn1`` ...).
"""
import numpy as np
import pytest
import torch


def _manifest(golden):
    z = golden('ref_detector.npz')
    keys = [str(k) for k in z['manifest.keys']]
    shapes = [tuple(int(d) for d in row if d >= 0) for row in z['manifest.shapes']]
    return keys, shapes


def _reference_checkpoint(golden, prefix='module.'):
    from oracle.weights import recipe_tensor
    keys, shapes = _manifest(golden)
    sd = {}
    for k, s in zip(keys, shapes):
        t = recipe_tensor(k, s, 21)
        sd[k] = torch.from_numpy(t) if t is not None else torch.zeros(s)
    # b0 backbone tensors of both ablation heads (efficientnet_pytorch naming)
    for head in ('sfe', 'sfe_cls'):
        sd[f'{head}.efficient_net._conv_stem.weight'] = torch.randn(32, 3, 3, 3)
        sd[f'{head}.efficient_net._bn0.running_mean'] = torch.randn(32)
        sd[f'{head}.efficient_net._bn0.num_batches_tracked'] = torch.tensor(7)
        sd[f'{head}.efficient_net._blocks.0._depthwise_conv.weight'] = torch.randn(32, 1, 3, 3)
    return {prefix + k: v for k, v in sd.items()}


def test_eval_py_strict_load_of_reference_checkpoint(golden, tmp_path):
    """eval.py:63-66: DeepfakeDetector(...); model.load_state_dict(torch.load(path))."""
    from network.model import DeepfakeDetector
    ckpt = _reference_checkpoint(golden)
    path = tmp_path / 'best_model.pth'
    torch.save(ckpt, path)
    model = DeepfakeDetector(in_channels=3, dama_dim=128)
    res = model.load_state_dict(torch.load(path, map_location='cpu', weights_only=True))
    assert not res.missing_keys and not res.unexpected_keys
    sd = model.state_dict()
    for k, v in ckpt.items():
        k = k[len('module.'):]
        assert k in sd, k
        assert torch.equal(sd[k].cpu(), v), k
    # the placeholders hold tensors only: nothing trainable was added
    n_train = sum(p.numel() for p in model.parameters() if p.requires_grad)
    fresh = sum(p.numel() for p in DeepfakeDetector(3, 128).parameters() if p.requires_grad)
    assert n_train == fresh
    # round trip: the product's state_dict loads strictly into a fresh product model
    again = DeepfakeDetector(3, 128)
    res = again.load_state_dict(sd)
    assert not res.missing_keys and not res.unexpected_keys


def test_strict_load_reports_real_mismatches(golden):
    from network.model import DeepfakeDetector
    ckpt = _reference_checkpoint(golden, prefix='')
    del ckpt['dama.gate_net.5.weight']
    ckpt['dama.not_a_key'] = torch.zeros(1)
    with pytest.raises(RuntimeError, match='gate_net.5.weight'):
        DeepfakeDetector(3, 128).load_state_dict(ckpt)


def test_load_reference_state_dict_drops_ablation_heads(golden):
    from network.model import DeepfakeDetector, load_reference_state_dict
    model = DeepfakeDetector(3, 128)
    missing, unexpected = load_reference_state_dict(model, _reference_checkpoint(golden))
    assert missing == [] and unexpected == []
    assert not any(k.startswith('sfe') for k in model.state_dict())


def test_product_key_set_is_reference_dynamic_subset(golden):
    """Every product state-dict key exists in the reference with the same shape."""
    from network.model import DeepfakeDetector
    keys, shapes = _manifest(golden)
    ref = dict(zip(keys, shapes))
    ours = DeepfakeDetector(3, 128).state_dict()
    for k, v in ours.items():
        assert k in ref, k
        assert tuple(v.shape) == ref[k], (k, tuple(v.shape), ref[k])
    missing = [k for k in ref if not k.startswith(('sfe.', 'sfe_cls.')) and k not in ours]
    assert missing == []


CURRICULUM = ((1, 10), (4, 10), (9, 10))


def _loss_inputs(z):
    return (torch.from_numpy(z['logits']), torch.from_numpy(z['space']), torch.from_numpy(z['freq']),
            torch.from_numpy(z['labels']))


@pytest.mark.parametrize('impl', ['product', 'product_device_weight', 'oracle'])
@pytest.mark.parametrize('epoch,maxe', CURRICULUM)
def test_combined_loss_vs_reference(golden, impl, epoch, maxe):
    """A14: BCEWithLogits(pos_weight) + curriculum-weighted orthogonality (train.py:55-91)."""
    from network import losses
    from oracle import model as om
    z = golden('ref_loss.npz')
    logits, space, freq, labels = _loss_inputs(z)
    lg, sp, fq = (t.clone().requires_grad_(True) for t in (logits, space, freq))
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5]))
    out = {'logits': lg, 'space': sp, 'freq': fq}
    if impl == 'product':
        loss, parts = losses.combined_loss(out, labels, crit, epoch, maxe)
    elif impl == 'product_device_weight':
        w = torch.tensor(losses.orth_weight(epoch, maxe))
        loss, parts = losses.combined_loss(out, labels, crit, 0, 0, weight=w)
    else:
        loss = om.combined_loss(out, labels, crit, epoch, maxe)
    loss.backward()
    tag = f'e{epoch}of{maxe}'
    torch.testing.assert_close(loss.detach(), torch.from_numpy(z[f'{tag}.loss']), rtol=1e-6, atol=1e-7)
    for name, t in (('logits', lg), ('space', sp), ('freq', fq)):
        g = t.grad if t.grad is not None else torch.zeros_like(t)
        torch.testing.assert_close(g, torch.from_numpy(z[f'{tag}.grad.{name}']), rtol=1e-5, atol=1e-8)


def test_orthogonal_loss_vs_reference(golden):
    from network import losses
    z = golden('ref_loss.npz')
    _, space, freq, _ = _loss_inputs(z)
    v = losses.orthogonal_loss(space, freq)
    np.testing.assert_allclose(float(v), float(z['orth']), rtol=1e-6)
    assert losses.orth_weight(1, 10) == 0.0 and losses.orth_weight(4, 10) == pytest.approx(0.4)
    assert losses.orth_weight(9, 10) == 1.0


def test_adam_launches_per_step_counts_both_forms():
    """The profilers' step-equivalent count (bench.py pmc_traffic): one table launch per
    parameter group, ceil(n / ADAM_MAX) launches per group in the per-48-tensor form."""
    from ewvit import _lib
    from ewvit.optim import Adam
    ps = [torch.nn.Parameter(torch.zeros(2)) for _ in range(2 * _lib.ADAM_MAX + 1)]
    frozen = torch.nn.Parameter(torch.zeros(2), requires_grad=False)
    opt = Adam([{'params': ps}, {'params': [frozen]}], lr=1e-3)
    assert opt.launches_per_step() == {'adam_table_kernel': 1, 'adam_multi_kernel': 3}
