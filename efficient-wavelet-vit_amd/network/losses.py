"""Training objective of the reference (train.py:55-91), used by bench.py and the
drop-in training step: BCEWithLogits(pos_weight) + curriculum-weighted
orthogonality between the space and freq features."""
import torch
from torch.nn import functional as F


def orthogonal_loss(space_feats, freq_feats):                              # train.py:55-67
    _, feat_dim = space_feats.shape
    s = F.normalize(space_feats, p=2, dim=1)
    f = F.normalize(freq_feats, p=2, dim=1)
    cov = torch.mm(s.T, f)
    off_diag = cov * (1 - torch.eye(feat_dim, device=cov.device))
    return torch.norm(off_diag, p='fro') ** 2 / (feat_dim * (feat_dim - 1))


def orth_weight(epoch, max_epochs):
    """The curriculum weight of the orthogonality term (train.py:76-86): 0 before 20 % of
    training, then a linear ramp reaching 1 at 70 %."""
    if epoch < 0.2 * max_epochs:
        return 0.0
    return min(1.0, (epoch - 0.2 * max_epochs) / (0.5 * max_epochs))


class _CombinedLoss(torch.autograd.Function):
    """ewvit_combined_loss: the loss and every input gradient in one launch on the GPU (the
    torch form below is ~40 small launches between the forward and the backward); the
    backward scales the saved gradients by the incoming one."""

    @staticmethod
    def forward(ctx, logits, labels, space, freq, pos_weight, weight, lam):
        from ewvit import _lib as L
        B, D = space.shape
        dev = space.device

        def on_dev(t, n):
            # labels / pos_weight / the curriculum weight may be CPU tensors (torch accepts a
            # 0-dim CPU weight): the kernel dereferences them, so they move to the GPU first
            return t.detach().to(device=dev, dtype=torch.float32).reshape(n).contiguous()
        lg = logits.detach().float().reshape(B).contiguous()
        lb = on_dev(labels, B)
        s, f = space.detach().float().contiguous(), freq.detach().float().contiguous()
        out = torch.empty(3, dtype=torch.float32, device=dev)
        dl, ds, df = torch.empty_like(lg), torch.empty_like(s), torch.empty_like(f)
        pw = on_dev(pos_weight, 1) if pos_weight is not None else None
        w = on_dev(weight, 1) if weight is not None else None
        L.require_gpu(lg, lb, s, f, pw, w)
        if any(t is not None and t.device != dev for t in (lg, lb, f, pw, w)):
            raise RuntimeError('combined_loss: inputs on different GPUs')
        L.call('ewvit_combined_loss', L.ptr(lg), L.ptr(lb), L.ptr(s), L.ptr(f), B, D, L.ptr(pw), L.ptr(w),
               float(lam), L.ptr(out), L.ptr(dl), L.ptr(ds), L.ptr(df), L.stream(out))
        ctx.save_for_backward(dl, ds, df)
        ctx.logit_shape = logits.shape
        total, parts = out[0], out[1:]
        ctx.mark_non_differentiable(parts)
        return total, parts

    @staticmethod
    def backward(ctx, g, _):
        dl, ds, df = ctx.saved_tensors
        dl, ds, df = torch._foreach_mul([dl, ds, df], g)
        return dl.view(ctx.logit_shape), None, ds, df, None, None, None


def _fused_ok(logits, labels, space, freq, criterion):
    return (logits.is_cuda and space.is_cuda and freq.is_cuda and logits.device == space.device == freq.device
            and torch.is_tensor(labels) and labels.numel() == logits.numel() and type(criterion) is torch.nn.BCEWithLogitsLoss and criterion.reduction == 'mean'
            and criterion.weight is None and (criterion.pos_weight is None or criterion.pos_weight.numel() == 1)
            and space.dim() == 2 and space.shape == freq.shape and logits.numel() == space.shape[0]
            and 1 <= space.shape[0] <= 64 and 4 * space.numel() + 2 * space.shape[0] + 16 <= 16384)


def combined_loss(outputs, labels, criterion, epoch, max_epochs, weight=None):  # train.py:69-91
    """weight: optional device tensor holding orth_weight(epoch, max_epochs), updated in place
    by the caller each epoch — the form a step replayed from a HIP graph needs (the
    epoch / max_epochs arguments are then ignored; a zero weight gives the reference's
    cls-only loss value and gradients).  On the GPU with the reference's criterion
    (BCEWithLogitsLoss, mean, scalar pos_weight) the whole objective is one ewvit launch."""
    logits = outputs['logits']
    if _fused_ok(logits, labels, outputs['space'], outputs['freq'], criterion):
        lam = 0.0 if weight is not None else orth_weight(epoch, max_epochs)
        total, parts = _CombinedLoss.apply(logits, labels, outputs['space'], outputs['freq'], criterion.pos_weight,
                                           weight, lam)
        orth = parts[1] if (weight is not None or lam != 0.0) else 0.0
        return total, {'cls_loss': parts[0], 'orth_loss': orth}
    labels = labels.view(-1, 1).float()
    cls_loss = criterion(logits, labels)
    if weight is not None:
        loss_orth = orthogonal_loss(outputs['space'], outputs['freq'])
        return cls_loss + weight * loss_orth, {'cls_loss': cls_loss.detach(), 'orth_loss': loss_orth.detach()}
    lam = orth_weight(epoch, max_epochs)
    if lam == 0.0:
        return cls_loss, {'cls_loss': cls_loss.detach(), 'orth_loss': 0.0}
    loss_orth = orthogonal_loss(outputs['space'], outputs['freq'])
    return cls_loss + lam * loss_orth, {'cls_loss': cls_loss.detach(), 'orth_loss': loss_orth.detach()}
