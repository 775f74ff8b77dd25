"""The N>1 path on CPU: world_size-2 `gloo` process group driving the same
ewvit.dist helpers bench.py uses (init from torchrun env, DDP wrap, video
sharding, max-over-ranks timing).  The model is the oracle's MWT (BatchNorm
inside, so per-replica statistics matter) — CPU-runnable; the product's HIP path
itself is exercised by the -m gpu tests.

Checks: DDP-averaged gradients == the gradient of the global-batch loss computed
the reference's DataParallel way (each replica's frames normalised with its own
BatchNorm statistics, loss = mean over all outputs); buffers of rank 0 broadcast;
timing reduced with MAX.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, REPO

WORLD = 2


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    from oracle import model as om
    torch.manual_seed(0)
    return om.MWT(3, 8, 2)


def _data():
    g = torch.Generator().manual_seed(5)
    return torch.randn(4, 2, 3, 16, 16, generator=g)       # [videos, frames, C, H, W]


def _worker(rank, port, q):
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from ewvit import dist as edist
    r, w, _ = edist.init_from_env('gloo')
    model = _model()
    net = edist.wrap(model)
    assert isinstance(net, torch.nn.parallel.DistributedDataParallel)
    x = edist.shard_videos(_data(), r, w)
    out = net(x.flatten(0, 1))
    out.mean().backward()
    grads = {n: p.grad.numpy().copy() for n, p in model.named_parameters()}
    t = edist.max_over_ranks(0.5 * (r + 1))
    # the next forward starts by broadcasting rank 0's buffers (eval: no further update)
    net.eval()
    with torch.no_grad():
        net(x.flatten(0, 1))
    q.put((r, grads, t, model.state_dict()["multiscale_fusion.1.running_mean"].numpy().copy()))
    edist.barrier()
    torch.distributed.destroy_process_group()


def test_ddp_gloo_world2_matches_dataparallel_semantics():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        r, g, t, rm = q.get(timeout=120)
        res[r] = (g, t, rm)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: one process, replicas run separately (own BN stats), loss = global mean
    ref = _model()
    x = _data()
    outs = [ref(x[2 * r:2 * r + 2].flatten(0, 1)) for r in range(WORLD)]
    torch.cat(outs).mean().backward()
    for n, p in ref.named_parameters():
        for r in range(WORLD):
            torch.testing.assert_close(torch.from_numpy(res[r][0][n]), p.grad, rtol=1e-5, atol=1e-6)
    assert res[0][1] == res[1][1] == 1.0                      # max over ranks
    torch.testing.assert_close(torch.from_numpy(res[0][2]), torch.from_numpy(res[1][2]))  # buffers broadcast


def _trainstep_worker(rank, port, q, accum=1, overlap=True, comm=None):
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from ewvit import dist as edist
    from ewvit.graph import TrainStep
    r, w, _ = edist.init_from_env('gloo')
    model = _model()
    if r == 1:                       # rank 1 starts from different BN buffers: the step broadcasts rank 0's
        for b in model.buffers():
            if b.dtype.is_floating_point:
                b.add_(3.0)
    x = edist.shard_videos(_data(), r, w)
    opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=0.5)
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    if accum == 1:
        def fl():
            return model(x.flatten(0, 1)).mean() / w
    else:                            # micro-batch k = frame k of every video
        def fl(k):
            return model(x[:, k]).mean() / w
    # 4 KB buckets: the MWT's ~40 gradients go out in many all-reduces, issued from the
    # post-accumulate hooks while backward is still running
    step = TrainStep(model, fl, opt, graph=False, bucket_mb=4 / 1024, accum_steps=accum, overlap=overlap,
                     grad_comm_dtype=comm)
    fired_in_backward = []
    orig_fire = step.buckets._fire

    def spy(b):
        fired_in_backward.append(b)
        return orig_fire(b)
    step.buckets._fire = spy
    at_finish = []
    orig_finish = step.buckets.finish

    def finish_spy():
        at_finish.append(len(fired_in_backward))      # buckets already issued while backward ran
        return orig_finish()
    step.buckets.finish = finish_spy
    step()                           # first step: initial layout, observes the gradient order
    assert fired_in_backward == list(range(len(fired_in_backward)))
    fired_in_backward.clear()
    for p, b in zip(model.parameters(), before.values()):    # replay the step from the same start
        p.data.copy_(b)
    step()                           # second step: the buffer re-cut in the observed order
    nb = len(step.buckets.buckets)
    first_order = list(step.buckets.order)
    grads = {n: p.grad.numpy().copy() for n, p in model.named_parameters()}
    delta = {n: (before[n] - p.detach()).numpy().copy() for n, p in model.named_parameters()}
    # every gradient is a view of the flat buffer after the step
    flat_ptrs = all(step.buckets.flat.data_ptr() <= p.grad.data_ptr() <
                    step.buckets.flat.data_ptr() + 4 * step.buckets.flat.numel() for p in model.parameters())
    if overlap:
        assert at_finish[-1] >= nb - 1, f'only {at_finish[-1]} of {nb} buckets issued during backward'
    q.put((r, grads, delta, nb, fired_in_backward, first_order, flat_ptrs))
    edist.barrier()
    torch.distributed.destroy_process_group()


def _run_trainstep(accum, overlap=True, comm=None):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_trainstep_worker, args=(r, port, q, accum, overlap, comm)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        r, g, d, nb, fired, order, flat_ptrs = q.get(timeout=120)
        res[r] = (g, d, nb, fired, order, flat_ptrs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(WORLD):
        g, d, nb, fired, order, flat_ptrs = res[r]
        assert nb > 4, 'expected several buckets'
        assert fired == list(range(nb)), 'buckets must be issued in order, each once'   # (no-ops when deferred)
        assert flat_ptrs, 'gradients must be views of the flat all-reduce buffer'
    assert res[0][4] == res[1][4], 'bucket layout agreed across ranks'
    return res


@pytest.mark.parametrize('overlap', [True, False])
def test_trainstep_gloo_world2_averages_gradients(overlap):
    """ewvit.graph.TrainStep (the bench's data-parallel step; eager mode on CPU):
    rank-0 buffers broadcast, bucketed all-reduces issued from the gradient hooks during
    backward in bucket order (overlap=False: the fallback's one all-reduce after backward),
    averaged gradients, identical updates — equal to the DataParallel-semantics gradient
    of the global batch."""
    res = _run_trainstep(1, overlap)
    ref = _model()
    x = _data()
    outs = [ref(x[2 * r:2 * r + 2].flatten(0, 1)) for r in range(WORLD)]
    torch.cat(outs).mean().backward()
    for n, p in ref.named_parameters():
        for r in range(WORLD):
            # TrainStep sums rank losses scaled by 1/world and divides the sum of
            # gradients by world: DataParallel's mean-over-all-outputs gradient / world
            torch.testing.assert_close(torch.from_numpy(res[r][0][n]) * WORLD, p.grad, rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(torch.from_numpy(res[r][1][n]), 0.5 * torch.from_numpy(res[r][0][n]),
                                       rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(torch.from_numpy(res[0][1][n]), torch.from_numpy(res[1][1][n]))


@pytest.mark.parametrize('overlap', [True, False])
def test_trainstep_gloo_world2_bf16_grad_allreduce(overlap):
    """grad_comm_dtype=torch.bfloat16 (opt-in): the buckets are rounded to bf16,
    all-reduced in bf16 and widened back into the fp32 buffer.  Equal to the fp32
    DataParallel-semantics gradient within the bf16 rounding of each rank's gradient and of
    the sum (relative 2^-7 of the gradient's scale), identical on both ranks."""
    res = _run_trainstep(1, overlap, torch.bfloat16)
    ref = _model()
    x = _data()
    outs = [ref(x[2 * r:2 * r + 2].flatten(0, 1)) for r in range(WORLD)]
    torch.cat(outs).mean().backward()
    worst = 0.0
    # (a floor on the scale: a bias feeding a train-mode BatchNorm has an exactly zero true
    # gradient, so its computed gradient is rounding noise in either dtype)
    gmax = max(float(p.grad.abs().max()) for p in ref.parameters())
    for n, p in ref.named_parameters():
        scale = max(float(p.grad.abs().max()), 1e-3 * gmax)
        for r in range(WORLD):
            g = torch.from_numpy(res[r][0][n]) * WORLD
            worst = max(worst, float((g - p.grad).abs().max()) / scale)
        assert np.array_equal(res[0][0][n], res[1][0][n])
    assert 0 < worst <= 2 ** -7, worst


def test_trainstep_gloo_world2_grad_accumulation():
    """accum_steps=2 (train.py:110-115: loss / accum_steps, backward per micro-batch, one
    optimizer step): the reduction runs once, after the last micro-batch, over the
    accumulated gradients."""
    res = _run_trainstep(2)
    ref = _model()
    x = _data()
    loss = 0
    for k in range(2):
        outs = [ref(x[2 * r:2 * r + 2, k]) for r in range(WORLD)]
        loss = loss + torch.cat(outs).mean() / 2
    loss.backward()
    for n, p in ref.named_parameters():
        for r in range(WORLD):
            torch.testing.assert_close(torch.from_numpy(res[r][0][n]) * WORLD, p.grad, rtol=1e-5, atol=1e-6)


def test_shard_videos_covers_batch_once():
    sys.path.insert(0, PKG)
    from ewvit import dist as edist
    x = torch.arange(10).view(10, 1)
    parts = [edist.shard_videos(x, r, 4) for r in range(4)]
    assert torch.equal(torch.cat(parts), x)


def _forced_worker(port, q):
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    torch.set_num_threads(1)
    import torch.distributed as tdist
    from ewvit.graph import TrainStep
    tdist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    model = _model()
    ref = _model()
    x = _data()[:2].flatten(0, 1)
    opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=0.5)
    step = TrainStep(model, lambda: model(x).mean(), opt, graph=False, bucket_mb=4 / 1024, force_collectives=True)
    fired = []
    orig = step.buckets._fire
    step.buckets._fire = lambda b: (fired.append(b), orig(b))[1]
    step()
    ref(x).mean().backward()
    ok = all(torch.allclose(p.grad, r.grad, rtol=1e-6, atol=1e-7) for p, r in zip(model.parameters(), ref.parameters()))
    q.put((fired, len(step.buckets.buckets), step.buckets.reduce, ok, step.describe()))
    tdist.destroy_process_group()


def test_force_collectives_world1_issues_bucket_allreduces():
    """TrainStep(force_collectives=True) in a world of one (the switch the GPU test uses to put
    RCCL calls in the captured step on a one-GPU box): the buckets are laid out and each one's
    all-reduce is issued, in order; the averaged gradient of one rank is its own gradient."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(_port(), q))
    p.start()
    fired, nb, reduce, ok, desc = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    # (the first step runs on the initial layout; the buffer is re-cut after it)
    assert reduce and nb > 4 and len(fired) > 4 and fired == list(range(len(fired))), (fired, nb)
    assert ok
    assert desc['world'] == 1 and desc['buckets'] == nb


def test_buffer_sync_skips_ablation_head_placeholders():
    """the checkpoint placeholders of the unused b0 heads (network/model.py
    _AblationHeadState) are never broadcast; BatchNorm running statistics are."""
    sys.path.insert(0, PKG)
    from ewvit.graph import BufferSync
    from network.model import _AblationHeadState
    m = torch.nn.Module()
    m.bn = torch.nn.BatchNorm2d(8)
    m.sfe = _AblationHeadState()
    m.sfe.inner = _AblationHeadState()
    m.sfe.inner.register_buffer('weight', torch.zeros(512, 1024))
    m.sfe.register_buffer('bias', torch.zeros(16))
    bs = BufferSync(m)
    # bn: running_mean + running_var (fp32) and num_batches_tracked (int64)
    assert bs.bytes == 2 * 8 * 4 + 8
    assert m.bn.running_mean.data_ptr() in {f.data_ptr() for f in bs.flats}
    assert m.sfe.inner.weight.numel() == 512 * 1024
