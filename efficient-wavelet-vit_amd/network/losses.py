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


def combined_loss(outputs, labels, criterion, epoch, max_epochs, weight=None):  # train.py:69-91
    """weight: optional device tensor holding orth_weight(epoch, max_epochs), updated in place
    by the caller each epoch — the form a step replayed from a HIP graph needs (the
    epoch / max_epochs arguments are then ignored; a zero weight gives the reference's
    cls-only loss value and gradients)."""
    logits = outputs['logits']
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
