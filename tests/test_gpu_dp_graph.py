"""The config-3 data-parallel step and the headline shape on the GPU.

* RCCL inside the captured step: a world-size-1 `nccl` process group (RCCL) with
  `TrainStep(force_collectives=True)`, which issues the bucket all-reduces and the BatchNorm
  buffer broadcast even at world 1 — the exact call sequence of `bench.py --gpus N`
  (reference train.py:249-251 `--multi-gpu`), recorded in ONE HIP graph.  The replays must
  equal the same steps issued eagerly, and the capture must not have fallen back to the
  split form.
* The bench shape: x = [8, 8, 3, 224, 224], batch_size=8 (one 64-frame `_process_frame`
  chunk, dama.py:179-186), bf16 autocast, the TrainStep graph: one replayed step against the
  same step issued eagerly from the same state (parameters, Adam moments, BatchNorm buffers,
  torch and ewvit RNG), every `pos_embedding[0:64]` row gets a gradient
  (sfe.py:126,158-159), BN counters advance once per BatchNorm call (3 for hf_conv's, which
  the DWT levels share).
* Adam after `load_state_dict`: a captured step keeps reading the loaded moments
  and the scheduler's lr.
"""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope='module')
def nccl_world1():
    from ewvit import dist as edist
    # before the group exists: no event cache (a captured collective's event must never be
    # handed to a later eager collective the watchdog polls), the flight recorder's
    # process-group status a global-mode capture waits on (ewvit.graph.retire_eager_collectives)
    edist.rccl_env()
    os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{_port()}', rank=0, world_size=1)
    assert dist.get_backend() == 'nccl'
    yield
    dist.destroy_process_group()


def _mwt_pair():
    from network.mwt import MWT
    torch.manual_seed(3)
    m = MWT(3, 64, 3).to(DEV).to(memory_format=torch.channels_last).train()
    return m, copy.deepcopy(m)


@pytest.mark.parametrize('mode', ['relaxed', 'global'])
def test_rccl_collectives_recorded_in_step_graph(nccl_world1, mode, monkeypatch):
    """Both capture modes need the NCCL watchdog's queue empty when the capture begins (its
    poll of an eager collective's event on the process group's stream, once that stream has
    joined the capture, fails with hipErrorCapturedEvent and aborts the process):
    TrainStep waits for its progress marker (ewvit.graph.retire_eager_collectives) — no sleep,
    no timing assumption."""
    monkeypatch.setenv('EWVIT_CAPTURE_MODE', mode)
    import ewvit
    from ewvit.graph import TrainStep
    a, b = _mwt_pair()
    x = torch.randn(4, 3, 64, 64, device=DEV)

    def make(m):
        opt = ewvit.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-4)

        def fl():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                return m(x).float().square().mean()
        return fl, opt
    fa, oa = make(a)
    fb, ob = make(b)
    # 64 KB buckets: the MWT's 0.2 M parameters go out in several all-reduces
    sa = TrainStep(a, fa, oa, graph=False, bucket_mb=1 / 16, force_collectives=True)
    for _ in range(6):
        sa()
    sb = TrainStep(b, fb, ob, graph=True, warmup=3, bucket_mb=1 / 16, force_collectives=True)
    d = sb.describe()
    assert d['launch'] == 'hip-graph' and 'capture_fallback' not in d, d
    assert d['overlap'].endswith('recorded in the step graph'), d
    assert d['buckets'] > 2, d
    assert sb.g2 is None                      # ONE graph: broadcast, fwd, bwd + all-reduces, Adam
    for _ in range(3):
        sb()
    torch.cuda.synchronize()
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(q, p, rtol=2e-4, atol=2e-5, msg=n)
    for (n, u), v in zip(a.named_buffers(), b.buffers()):
        torch.testing.assert_close(v, u, rtol=2e-4, atol=2e-5, msg=n)
    # the gradients the optimizer read are views of the all-reduced flat buffer
    flat = sb.buckets.flat
    assert all(flat.data_ptr() <= p.grad.data_ptr() < flat.data_ptr() + 4 * flat.numel()
               for p in b.parameters() if p.requires_grad)
    sa.close()
    sb.close()                                # the RCCL-holding graph released while the group lives


def test_capture_failure_raises_without_opt_in(nccl_world1, monkeypatch):
    """A capture failure must fail the step (and a bench run), not silently time the split
    form; EWVIT_GRAPH_SPLIT_FALLBACK=1 opts in to the fallback, which describe() names."""
    import ewvit
    from ewvit import graph as eg
    a, _ = _mwt_pair()
    x = torch.randn(2, 3, 32, 32, device=DEV)
    opt = ewvit.optim.Adam([p for p in a.parameters() if p.requires_grad], lr=1e-3)

    def fl():
        with torch.autocast('cuda', dtype=torch.bfloat16):
            return a(x).float().square().mean()

    def boom(self, warmup):
        raise RuntimeError('simulated capture failure')
    monkeypatch.setattr(eg.TrainStep, '_capture', boom)
    monkeypatch.delenv('EWVIT_GRAPH_SPLIT_FALLBACK', raising=False)
    with pytest.raises(RuntimeError, match='simulated'):
        eg.TrainStep(a, fl, opt, graph=True, force_collectives=True)
    monkeypatch.setenv('EWVIT_GRAPH_SPLIT_FALLBACK', '1')
    s = eg.TrainStep(a, fl, opt, graph=True, force_collectives=True)
    d = s.describe()
    assert 'simulated' in d['capture_fallback'] and d['overlap'] == 'one all-reduce between two graphs'
    s()
    torch.cuda.synchronize()
    s.close()


def _snapshot(step):
    from ewvit import _lib
    m, opt = step.model, step.opt
    st = {'params': [p.detach().clone() for p in m.parameters()],
          'buffers': [b.detach().clone() for b in m.buffers()],
          'opt': [{k: v.detach().clone() for k, v in opt.state[p].items()} for p in step.params if p in opt.state],
          'rng': torch.cuda.get_rng_state(),
          'ewvit_rng': _lib.rng_offset(torch.device(DEV)).clone()}
    return st


def _restore(step, st):
    from ewvit import _lib
    m, opt = step.model, step.opt
    with torch.no_grad():
        for p, v in zip(m.parameters(), st['params']):
            p.copy_(v)
        for b, v in zip(m.buffers(), st['buffers']):
            b.copy_(v)
        for p, saved in zip([p for p in step.params if p in opt.state], st['opt']):
            for k, v in saved.items():
                opt.state[p][k].copy_(v)
        _lib.rng_offset(torch.device(DEV)).copy_(st['ewvit_rng'])
    torch.cuda.set_rng_state(st['rng'])
    torch.cuda.synchronize()


def test_bench_shape_graph_step_equals_eager(nccl_world1):
    """config 2/3 at its own size: DeepfakeDetector(3, 128, batch_size=8) on x [8, 8, 3, 224,
    224] (one 64-frame chunk), bf16 autocast, combined_loss with the orthogonality term,
    ewvit Adam, the RCCL bucket all-reduces forced on — one graph replay vs the same step
    issued eagerly from the same state."""
    import bench
    step = bench.build_step(torch.device(DEV), 64, 0, graph=True, config=2, force_collectives=True)
    d = step.describe()
    assert d['launch'] == 'hip-graph' and d['overlap'].endswith('recorded in the step graph'), d
    model = step.model
    nbt = [(n, b) for n, b in model.named_buffers() if n.endswith('num_batches_tracked')]
    assert nbt
    snap = _snapshot(step)
    nbt0 = [int(b) for _, b in nbt]

    loss_g = float(step())
    torch.cuda.synchronize()
    assert torch.isfinite(torch.tensor(loss_g))
    grads_g = step.buckets.flat.clone()
    params_g = [p.detach().clone() for p in model.parameters()]
    bufs_g = [b.detach().clone() for b in model.buffers()]
    d_g = [int(b) - v for (_, b), v in zip(nbt, nbt0)]
    # one chunk: every BatchNorm of the step runs once, except hf_conv's, shared by the 3 DWT
    # levels (reference mwt.py:47-65,108: called once per level); DeepfakeDetector.mwt is
    # unused in 'dynamic' mode (model.py:37-58) and never runs
    want = [3 if '.mwt.hf_conv.' in n else (1 if n.startswith('dama.') else 0) for n, _ in nbt]
    assert d_g == want, [(n, a, b) for (n, _), a, b in zip(nbt, d_g, want) if a != b]

    _restore(step, snap)
    # the replay's dropout / drop-path launches use host seeds drawn at capture (ewvit.ops._seed,
    # mixed with the device step counter restored above): the eager step draws the same ones
    torch.set_rng_state(step.capture_cpu_rng)
    loss_e = float(step._eager())
    torch.cuda.synchronize()
    grads_e = step.buckets.flat.clone()
    assert [int(b) - v for (_, b), v in zip(nbt, nbt0)] == want
    assert loss_e == pytest.approx(loss_g, rel=1e-5, abs=1e-6)
    cos = torch.nn.functional.cosine_similarity(grads_g.double(), grads_e.double(), dim=0)
    err = float((grads_g - grads_e).abs().max() / grads_e.abs().max())
    print(f'bench-shape graph vs eager: loss {loss_g:.6f}/{loss_e:.6f}, grad cos {float(cos):.8f}, '
          f'max err {err:.3e} of scale')
    assert float(cos) > 0.99999 and err < 1e-4
    for (n, p), q in zip(model.named_parameters(), params_g):
        torch.testing.assert_close(q, p.detach(), rtol=1e-5, atol=1e-7, msg=n)
    for (n, b), v in zip(model.named_buffers(), bufs_g):
        torch.testing.assert_close(v, b, rtol=1e-5, atol=1e-6, msg=n)

    # every frame position of the chunk reaches the CLS/patch tokens through pos_embedding[0:64]
    sfe = model.dama.sfe
    pe = sfe.pos_embedding
    assert pe.shape[0] == 64
    g = pe.grad
    assert g is not None and g.shape == pe.shape
    rows = g.reshape(64, -1).abs().amax(1)
    assert bool((rows > 0).all()), f'rows without gradient: {(rows == 0).nonzero().flatten().tolist()}'
    step.close()


def test_adam_load_state_dict_after_capture_follows_loaded_state():
    """torch's load_state_dict replaces the param_group dicts and the state
    tensors.  ewvit Adam copies the loaded moments into the tensors the graph reads and keys
    its lr scalars by group index, so a step captured before the load follows the loaded
    moments, the loaded lr and the scheduler after it — like the eager twin."""
    import ewvit
    from ewvit.graph import TrainStep
    a, b = _mwt_pair()
    x = torch.randn(4, 3, 64, 64, device=DEV)

    def make(m):
        opt = ewvit.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=3e-3, weight_decay=1e-4)

        def fl():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                return m(x).float().square().mean()
        return fl, opt
    fa, oa = make(a)
    fb, ob = make(b)
    sa = TrainStep(a, fa, oa, graph=False)
    for _ in range(3):
        sa()
    sb = TrainStep(b, fb, ob, graph=True, warmup=3)

    def reload(opt):
        sd = copy.deepcopy(opt.state_dict())
        sd['param_groups'][0]['lr'] = 1e-2
        for s in sd['state'].values():
            s['exp_avg'] = torch.zeros_like(s['exp_avg'])
            s['step'] = s['step'].cpu()       # a torch checkpoint keeps the step on the host
        opt.load_state_dict(sd)
        return torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=4)
    ra, rb = reload(oa), reload(ob)
    for _ in range(3):
        sa()
        ra.step()
        sb()
        rb.step()
    torch.cuda.synchronize()
    assert oa.param_groups[0]['lr'] < 1e-2 * 0.9
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(q, p, rtol=2e-4, atol=2e-5, msg=n)
