"""GPU parity of the fused combined_loss (ewvit_combined_loss; reference train.py:55-91): the
loss value and the logits / space / freq gradients against the reference's own outputs
(tests/golden/ref_loss.npz) and against the torch formulation of network/losses.py on the
same device, at the curriculum points, with a device weight, without pos_weight, and for a
zero-norm row (F.normalize's eps branch).  fp32 throughout: bounds 2e-6 relative on the
value, 2e-5 relative on gradients (a different summation order of the same fp32 terms; per
row, 1e-5 of the row's largest gradient absolute, x sqrt(D / 128) past D = 128: g - u (u . g)
cancels, and its rounding grows with the length of the D-term sums)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


class _TorchBCE(torch.nn.BCEWithLogitsLoss):
    """a subclass: combined_loss keeps its torch formulation for it (the comparison path)"""


def _run(impl_crit, logits, space, freq, labels, epoch=1, maxe=1, weight=None):
    from network import losses
    lg, sp, fq = (t.clone().to(DEV).requires_grad_(True) for t in (logits, space, freq))
    out = {'logits': lg, 'space': sp, 'freq': fq}
    loss, parts = losses.combined_loss(out, labels.to(DEV), impl_crit, epoch, maxe, weight=weight)
    loss.backward()
    return loss.detach().cpu(), parts, [t.grad.cpu() if t.grad is not None else torch.zeros_like(t).cpu()
                                        for t in (lg, sp, fq)]


@pytest.mark.parametrize('epoch,maxe', [(1, 10), (4, 10), (9, 10)])
def test_fused_loss_vs_reference_golden(golden, epoch, maxe):
    from network import losses
    z = golden('ref_loss.npz')
    logits, space, freq = (torch.from_numpy(z[k]) for k in ('logits', 'space', 'freq'))
    labels = torch.from_numpy(z['labels'])
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5], device=DEV))
    assert losses._fused_ok(logits.to(DEV), labels, space.to(DEV), freq.to(DEV), crit)
    tag = f'e{epoch}of{maxe}'
    for weight in (None, torch.tensor(losses.orth_weight(epoch, maxe), device=DEV)):
        loss, parts, grads = _run(crit, logits, space, freq, labels, epoch, maxe, weight)
        torch.testing.assert_close(loss, torch.from_numpy(z[f'{tag}.loss']), rtol=2e-6, atol=1e-7)
        for name, g in zip(('logits', 'space', 'freq'), grads):
            torch.testing.assert_close(g, torch.from_numpy(z[f'{tag}.grad.{name}']), rtol=2e-5, atol=1e-9)


@pytest.mark.parametrize('B,D,pw', [(8, 128, 0.5), (3, 64, None), (16, 192, 2.0), (1, 8, 0.5),
                                         (40, 80, 0.5), (4, 512, 1.5), (32, 96, None)])
def test_fused_loss_vs_torch(B, D, pw):
    g = torch.Generator().manual_seed(B * 131 + D)
    logits = torch.randn(B, 1, generator=g) * 3
    space, freq = torch.randn(B, D, generator=g), torch.randn(B, D, generator=g) * 0.1
    labels = (torch.rand(B, generator=g) > 0.5).float()
    if B > 2:
        space[1].zero_()                    # ||x|| < eps: the gradient is g / eps
    pwt = None if pw is None else torch.tensor([pw], device=DEV)
    w = torch.tensor(0.7, device=DEV)
    ref = _run(_TorchBCE(pos_weight=pwt), logits, space, freq, labels, weight=w)
    got = _run(torch.nn.BCEWithLogitsLoss(pos_weight=pwt), logits, space, freq, labels, weight=w)
    torch.testing.assert_close(got[0], ref[0], rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(got[1]['cls_loss'].cpu(), ref[1]['cls_loss'].cpu(), rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(got[1]['orth_loss'].cpu(), ref[1]['orth_loss'].cpu(), rtol=2e-5, atol=1e-9)
    for a, b in zip(got[2], ref[2]):
        for r in range(B):                  # per row: the zero row's gradient is ~1e12 larger
            scale = float(b[r].abs().max()) + 1e-30
            torch.testing.assert_close(a[r], b[r], rtol=2e-5, atol=1e-5 * max(1.0, (D / 128) ** 0.5) * scale)


def test_fused_loss_grad_scale_and_graph():
    """the backward scales the saved gradients by the incoming one; capturable"""
    from network import losses
    g = torch.Generator().manual_seed(3)
    logits, space, freq = torch.randn(8, 1, generator=g), torch.randn(8, 128, generator=g), torch.randn(8, 128,
                                                                                                        generator=g)
    labels = (torch.rand(8, generator=g) > 0.5).float().to(DEV)
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5], device=DEV))
    sp = space.to(DEV).requires_grad_(True)
    out = {'logits': logits.to(DEV), 'space': sp, 'freq': freq.to(DEV)}
    loss, _ = losses.combined_loss(out, labels, crit, 9, 10)
    (3.0 * loss).backward()
    sp2 = space.to(DEV).requires_grad_(True)
    loss2, _ = losses.combined_loss({'logits': logits.to(DEV), 'space': sp2, 'freq': freq.to(DEV)}, labels, crit, 9,
                                    10)
    loss2.backward()
    torch.testing.assert_close(sp.grad, 3.0 * sp2.grad, rtol=1e-6, atol=0)
    # one launch replayed from a HIP graph follows a device weight written between replays
    w = torch.tensor(0.0, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            lv, _ = losses.combined_loss(out, labels, crit, 0, 0, weight=w)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            lv, parts = losses.combined_loss(out, labels, crit, 0, 0, weight=w)
    torch.cuda.current_stream().wait_stream(s)
    w.fill_(1.0)
    graph.replay()
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(lv), float(parts['cls_loss']) + float(parts['orth_loss']), rtol=1e-6)
    assert float(parts['orth_loss']) > 0


def test_fused_loss_host_operands():
    """labels, pos_weight and a 0-dim curriculum weight given as CPU tensors (torch
    accepts them) go to the GPU before the launch — the kernel must never read a host
    address.  Same values as the all-device call."""
    from network import losses
    g = torch.Generator().manual_seed(11)
    logits, space, freq = torch.randn(8, 1, generator=g), torch.randn(8, 128, generator=g), torch.randn(8, 128,
                                                                                                        generator=g)
    labels = (torch.rand(8, generator=g) > 0.5).float()
    dev_crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5], device=DEV))
    host_crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor(0.5))
    ref = _run(dev_crit, logits, space, freq, labels.to(DEV), weight=torch.tensor(0.7, device=DEV))
    out = {'logits': logits.to(DEV).requires_grad_(True), 'space': space.to(DEV).requires_grad_(True),
           'freq': freq.to(DEV).requires_grad_(True)}
    assert losses._fused_ok(out['logits'], labels, out['space'], out['freq'], host_crit)
    loss, _ = losses.combined_loss(out, labels, host_crit, 1, 1, weight=torch.tensor(0.7))
    loss.backward()
    torch.cuda.synchronize()
    torch.testing.assert_close(loss.detach().cpu(), ref[0], rtol=0, atol=0)
    for t, r in zip((out['logits'], out['space'], out['freq']), ref[2]):
        torch.testing.assert_close(t.grad.cpu(), r, rtol=0, atol=0)
