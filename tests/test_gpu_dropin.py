"""The drop-in contract with the reference's own training loop.

* fp32 callers: the reference trains in fp32, no autocast, default memory format
  (train.py:16, 93-140).  The modules compute in bf16 anyway (network.bf16_compute enters
  autocast when the caller has not) — so the reference's train_epoch body, restated statement
  for statement below, runs with NO library convolution, BatchNorm or GEMM inside the model
  (a dispatch-mode recorder sees every aten op the forward issues), returns fp32 outputs, and
  takes the same kernels as an autocast caller.
* threads: `--multi-gpu` is nn.DataParallel (train.py:249-251), which runs each replica's
  forward in its own Python thread.  Two replicas driven concurrently from two threads on two
  streams of one GPU must produce bit-for-bit the outputs, gradients and BatchNorm statistics
  of the same two replicas run one after the other (the per-call state — the branch grid cap,
  the BatchNorm backward links, the skip links, the weight packs — is per thread).
"""
import copy
import threading

import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode

pytestmark = pytest.mark.gpu
DEV = 'cuda'

# aten ops a library conv / BatchNorm / GEMM would show up as
BANNED = ('convolution', 'conv2d', 'cudnn', 'miopen', 'batch_norm', 'addmm', 'linear', 'bmm', 'matmul',
          'aten.mm.', 'baddbmm', 'layer_norm', 'upsample')


class _Ops(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.names = set()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        self.names.add(str(func))
        return func(*args, **(kwargs or {}))


def _no_stochastic(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        if hasattr(mod, 'sd_prob'):
            mod.sd_prob = 0.0
    return m


def _orthogonal_loss(space_feats, freq_feats):            # train.py:55-67, verbatim semantics
    _, feat_dim = space_feats.shape
    space_feats = torch.nn.functional.normalize(space_feats, p=2, dim=1)
    freq_feats = torch.nn.functional.normalize(freq_feats, p=2, dim=1)
    cov = torch.mm(space_feats.T, freq_feats)
    diag_mask = torch.eye(feat_dim).to(cov.device)
    off_diag = cov * (1 - diag_mask)
    return torch.norm(off_diag, p='fro') ** 2 / (feat_dim * (feat_dim - 1))


def _combined_loss(outputs, labels, criterion, epoch, max_epochs):   # train.py:69-91
    logits = outputs['logits']
    labels = labels.view(-1, 1).float()
    if epoch < 0.2 * max_epochs:
        cls_loss = criterion(logits, labels)
        return cls_loss, {'cls_loss': cls_loss.item(), 'orth_loss': 0.0}
    cls_loss = criterion(logits, labels)
    loss_orth = _orthogonal_loss(outputs['space'], outputs['freq'])
    lambda_orth = min(1.0, (epoch - 0.2 * max_epochs) / (0.5 * max_epochs))
    return cls_loss + lambda_orth * loss_orth, {'cls_loss': cls_loss.item(), 'orth_loss': loss_orth.item()}


def test_reference_train_epoch_fp32_runs_no_library_ops():
    from network.model import DeepfakeDetector
    torch.manual_seed(0)
    device = torch.device(DEV)
    batch_size = 4
    model = DeepfakeDetector(in_channels=3, dama_dim=128, batch_size=batch_size).to(device)   # train.py:243-247
    criterion = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5]).to(device))        # train.py:270-272
    optimizer = torch.optim.Adam(model.parameters(), lr=1e-4, weight_decay=1e-4)            # train.py:273
    g = torch.Generator().manual_seed(1)
    dataloader = [(torch.randn(2, 4, 3, 224, 224, generator=g), torch.tensor([0, 1])) for _ in range(2)]
    w0 = model.dama.mwt.multiscale_fusion[0].weight.detach().clone()

    # train_epoch (train.py:93-140), accum_steps=2, epoch 1 of 1 (orthogonality term on)
    accum_steps, epoch, max_epochs = 2, 1, 1
    model.train()
    running_loss = 0.0
    preds_all, labels_all = [], []
    optimizer.zero_grad()
    seen = set()
    for i, (frames, labels) in enumerate(dataloader):
        frames, labels = frames.to(device), labels.to(device)
        rec = _Ops()
        with rec:
            outputs = model(frames, batch_size=batch_size, ablation='dynamic')
        seen |= rec.names
        assert all(v.dtype == torch.float32 for v in outputs.values()), {k: v.dtype for k, v in outputs.items()}
        loss, losses = _combined_loss(outputs, labels, criterion, epoch, max_epochs)
        orig_loss = loss
        loss = loss / accum_steps
        loss.backward()
        if (i + 1) % accum_steps == 0:
            optimizer.step()
            optimizer.zero_grad()
        running_loss += orig_loss.item() * frames.size(0)
        preds = torch.sigmoid(outputs['logits']).squeeze(1).detach().cpu().numpy()
        preds_all.extend(preds)
        labels_all.extend(labels.cpu().numpy())
    bad = sorted(n for n in seen if n.startswith('aten.') and any(b in n for b in BANNED))
    assert not bad, bad
    assert any(n.startswith('ewvit.') for n in seen), sorted(seen)[:20]     # the custom ops ran
    assert len(preds_all) == 4 and torch.isfinite(torch.tensor(running_loss))
    assert not torch.equal(model.dama.mwt.multiscale_fusion[0].weight, w0)  # the optimizer stepped


def _step(model, x, stream, out):
    with torch.cuda.stream(stream):
        r = model(x, 8, 'dynamic')
        loss = r['logits'].float().square().sum() + r['space'].float().square().mean() + r['freq'].float().mean()
        loss.backward()
    stream.synchronize()
    out['y'] = {k: v.detach().clone() for k, v in r.items()}
    out['g'] = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    out['b'] = {n: b.detach().clone() for n, b in model.named_buffers()}


def test_two_replica_threads_match_serial():
    from network.model import DeepfakeDetector
    torch.manual_seed(3)
    base = _no_stochastic(DeepfakeDetector(3, 128, batch_size=8)).to(DEV).train()
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(1, 8, 3, 224, 224, generator=g).to(DEV) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()

    serial = [{}, {}]
    reps = [copy.deepcopy(base) for _ in range(2)]
    for i in range(2):
        _step(reps[i], xs[i], streams[i], serial[i])

    conc = [{}, {}]
    reps = [copy.deepcopy(base) for _ in range(2)]
    errs = []

    def worker(i):
        try:
            _step(reps[i], xs[i], streams[i], conc[i])
        except Exception as e:          # noqa: BLE001 — reported by the main thread
            errs.append(e)
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errs, errs
    for i in range(2):
        for part in ('y', 'g', 'b'):
            a, b = serial[i][part], conc[i][part]
            assert a.keys() == b.keys()
            diff = [k for k in a if not torch.equal(a[k], b[k])]
            assert not diff, (i, part, diff[:8])
    assert not torch.equal(serial[0]['y']['fused'], serial[1]['y']['fused'])
