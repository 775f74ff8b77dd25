"""HIP-graph replay of the training step (ewvit/graph.py) on the GPU: the replayed
iteration must equal the same iteration issued eagerly, and ewvit dropout must draw
a fresh mask on every replay (device step counter, csrc/common.h step_seed)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _mwt_pair():
    from network.mwt import MWT
    torch.manual_seed(3)
    m = MWT(3, 64, 3).to(DEV).to(memory_format=torch.channels_last).train()
    return m, copy.deepcopy(m)


def test_trainstep_graph_replay_equals_eager():
    from ewvit.graph import TrainStep
    a, b = _mwt_pair()
    x = torch.randn(4, 3, 64, 64, device=DEV)

    def make(m):
        opt = torch.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=1e-3, fused=True,
                               capturable=True)

        def fl():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                return m(x).float().square().mean()
        return fl, opt
    fa, oa = make(a)
    fb, ob = make(b)
    sa = TrainStep(a, fa, oa, graph=False)
    for _ in range(6):                       # 3 warm-up iterations + 3 replays on the graph side
        sa()
    sb = TrainStep(b, fb, ob, graph=True, warmup=3)
    for _ in range(3):
        sb()
    torch.cuda.synchronize()
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(q, p, rtol=2e-4, atol=2e-5, msg=n)
    for (n, u), v in zip(a.named_buffers(), b.buffers()):
        torch.testing.assert_close(v, u, rtol=2e-4, atol=2e-5, msg=n)
    assert float(sb.loss) == pytest.approx(float(sa.loss), rel=1e-3)


def _adam_pair(sched_steps_after=3, accum=1):
    """Eager vs graph TrainStep with ewvit.optim.Adam (the bench's optimizer): 3 steps at
    the initial lr, then 3 steps each followed by a CosineAnnealingLR step."""
    import ewvit
    from ewvit.graph import TrainStep
    a, b = _mwt_pair()
    xs = torch.randn(accum, 4, 3, 64, 64, device=DEV)

    def make(m):
        opt = ewvit.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=3e-3, weight_decay=1e-4)
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=4)

        def fl(k=0):
            with torch.autocast('cuda', dtype=torch.bfloat16):
                return m(xs[k]).float().square().mean()
        return fl, opt, sched
    fa, oa, sa_ = make(a)
    fb, ob, sb_ = make(b)
    sa = TrainStep(a, fa, oa, graph=False, accum_steps=accum)
    for _ in range(3):
        sa()
    for _ in range(3):
        sa()
        sa_.step()
    sb = TrainStep(b, fb, ob, graph=True, warmup=3, accum_steps=accum)      # 3 steps run while capturing
    for _ in range(3):
        sb()
        sb_.step()
    torch.cuda.synchronize()
    assert oa.param_groups[0]['lr'] < 3e-3 * 0.9            # the schedule moved the lr
    return a, b, sa, sb


def test_trainstep_graph_single_launch_adam_equals_eager():
    """ewvit Adam inside the captured step: the capture launches the one-launch form on a
    table allocated before the capture and filled after it (Adam.finish_capture); the replays
    match the same steps run eagerly"""
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
    sa = TrainStep(a, fa, oa, graph=False)
    for _ in range(6):
        sa()
    sb = TrainStep(b, fb, ob, graph=True, warmup=3)
    # the captured table belongs to the graph (freed with it), none kept by the optimizer
    assert len(sb.g._ewvit_adam_tables) == 1 and not getattr(ob, '_fill_after_capture', [])
    assert not getattr(ob, '_table_keep', [])
    for _ in range(3):
        sb()
    torch.cuda.synchronize()
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(q, p, rtol=2e-4, atol=2e-5, msg=n)


def test_trainstep_graph_follows_lr_schedule():
    """a replayed step must read the scheduler's lr (device scalar refreshed
    before each replay), not the lr baked in at capture."""
    a, b, sa, sb = _adam_pair()
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(q, p, rtol=2e-4, atol=2e-5, msg=n)
    assert float(sb.loss) == pytest.approx(float(sa.loss), rel=1e-3)


def test_trainstep_graph_grad_accumulation():
    """accum_steps=2 recorded in the graph (train.py:110-115) equals the eager loop."""
    a, b, sa, sb = _adam_pair(accum=2)
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(q, p, rtol=2e-4, atol=2e-5, msg=n)


def test_dropout_mask_changes_per_replay():
    import ewvit
    x = torch.randn(64, 128, device=DEV)
    w = torch.randn(96, 128, device=DEV)
    out = torch.empty(64, 96, device=DEV)

    def body():
        ewvit._lib.rng_advance(x.device)
        out.copy_(ewvit.linear(x, w, drop_p=0.5))
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    g.replay()
    m1 = (out == 0).clone()
    g.replay()
    m2 = (out == 0).clone()
    assert 0.4 < float(m1.float().mean()) < 0.6
    assert not torch.equal(m1, m2)


def test_grad_slots_adopted_and_multi_use():
    """ewvit.grads slots: a conv / linear weight used once gets its gradient written into the
    flat buffer and ADOPTED by AccumulateGrad (no clone: the gradient's storage is the slot's
    when the first post-accumulate hook sees it); a weight used twice in one forward gets the
    sum of both uses: the first use in backward order writes the slot, the second a fresh
    tensor, and ewvit.grads adds it in at the end of the backward pass (no autograd add, no copy
    into the slot).  The backward runs on autograd's device thread: the ops carry the forward
    thread's step id to it (ewvit.grads.note_use)."""
    from ewvit import grads, ops
    from ewvit.conv import conv2d
    from ewvit.graph import GradBuckets
    torch.manual_seed(5)
    w1 = torch.nn.Parameter(torch.randn(64, 32, 3, 3, device=DEV) * 0.1)
    w2 = torch.nn.Parameter(torch.randn(64, 64, 1, 1, device=DEV) * 0.1)     # used twice
    lw = torch.nn.Parameter(torch.randn(48, 64, device=DEV) * 0.1)
    lb = torch.nn.Parameter(torch.randn(48, device=DEV) * 0.1)
    params = [w1, w2, lw, lb]
    x = torch.randn(4, 32, 16, 16, device=DEV).to(memory_format=torch.channels_last)

    def fwd():
        y = conv2d(x, w1, None, 1)
        y = conv2d(conv2d(y, w2, None, 1), w2, None, 1)
        t = y.float().mean((2, 3))
        return ops.linear(t, lw, lb).square().sum()

    fwd().backward()                         # reference gradients, no slots
    ref = [p.grad.clone() for p in params]
    for p in params:
        p.grad = None
    stolen = {}
    for i, p in enumerate(params):           # registered before GradBuckets' hooks: runs first
        p.register_post_accumulate_grad_hook(
            lambda q, i=i: stolen.__setitem__(i, q.grad.data_ptr()) if q.grad is not None else None)
    gb = GradBuckets(params)
    try:
        gb.begin()
        grads.begin_step()
        fwd().backward()
        torch.cuda.synchronize()
    finally:
        gb.remove()
    for i, (p, r) in enumerate(zip(params, ref)):
        assert p.grad.data_ptr() == gb.views[i].data_ptr()
        torch.testing.assert_close(p.grad, r, rtol=1e-5, atol=1e-6)
    for i in (0, 1, 2, 3):                   # written in place (two uses: summed in place), no clone
        assert stolen[i] == gb.views[i].data_ptr(), i


@pytest.mark.parametrize('graph', [False, True])
def test_trainstep_early_params_same_update(graph):
    """TrainStep(early_params=...): the parameters whose gradients are final early get their
    Adam update on a side stream as soon as the last of them is accumulated, the rest after the
    backward — the same bits as one optimizer step (ewvit.optim.Adam is per-parameter), eager and
    replayed; the early step really fires before the end of the backward pass."""
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
    import ewvit.graph as egraph
    import os
    os.environ['EWVIT_EARLY_STEP'] = '1'
    sa = TrainStep(a, fa, oa, graph=graph, warmup=2)
    # the layers nearest the loss finish their gradients first: the last half of the parameters
    pb = [p for p in b.parameters() if p.requires_grad]
    try:
        sb = TrainStep(b, fb, ob, graph=graph, warmup=2, early_params=pb[len(pb) // 2:])
    finally:
        del os.environ['EWVIT_EARLY_STEP']
    del egraph
    assert sb._early is not None and ob.launches_per_step()['adam_table_kernel'] == 2
    for _ in range(3):
        sa()
        sb()
    torch.cuda.synchronize()
    assert sb._early['fired']                       # issued from the backward pass, not the fallback
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(p, q), n
    for (n, u), v in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(u, v), n
    sb.close()
    assert not any(getattr(p, '_ewvit_early', False) for p in b.parameters())
