"""ewvit.grads on the CPU: gradient slots and the deferred sum of a parameter used more than
once in a step (DAMA's frame chunks, dama.py:179-186).  A toy op follows the product ops'
protocol — ``note_use`` in the forward, ``grad_out`` for the weight gradient's output,
``give`` for what autograd receives — and the result must equal autograd's own summation:
the gradient values, ``param.grad`` living in the flat slot, and the post-accumulate hook
(the data-parallel bucket hook) running once per parameter with the gradient in place."""
import pytest
import torch

from ewvit import grads


class _Scale(torch.autograd.Function):
    """y = x * w (w [D]); dW written into grad_out's tensor like the product's wgrad kernels."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.gen = grads.note_use(w)
        ctx.params = (w,)
        ctx.save_for_backward(x)
        return x * w

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        w = ctx.params[0]
        dw = grads.grad_out(w, ctx.gen)
        dw.copy_((g * x).sum(0))
        return g * w.detach(), grads.give(w, dw, ctx.gen)


def _run(uses, defer, slot, accumulate=False, seed=0):
    torch.manual_seed(seed)
    D = 8
    w = torch.nn.Parameter(torch.randn(D))
    v = torch.nn.Parameter(torch.randn(D))          # a single-use parameter beside it
    flat = torch.zeros(2 * D)
    if slot:
        grads.set_slot(w, flat, 0)
        grads.set_slot(v, flat, D)
    calls = []
    for p in (w, v):
        p.register_post_accumulate_grad_hook(lambda t, p=p: calls.append((p is w, None if t.grad is None else t.grad.clone())))
    if accumulate:
        w.grad = torch.ones(D)
    xs = [torch.randn(4, D) for _ in range(uses)]
    old = grads.DEFER
    grads.DEFER = defer
    try:
        grads.begin_step()
        loss = sum((_Scale.apply(x, w) ** 2).sum() for x in xs) + (_Scale.apply(xs[0], v) ** 3).sum()
        loss.backward()
    finally:
        grads.DEFER = old
    return w, v, flat, calls


@pytest.mark.parametrize('uses', [1, 2, 3])
@pytest.mark.parametrize('slot', [False, True])
def test_deferred_sum_equals_autograd(uses, slot):
    wa, va, flat, calls = _run(uses, True, slot)
    wb, vb, _, _ = _run(uses, False, slot)
    torch.testing.assert_close(wa.grad, wb.grad, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(va.grad, vb.grad, rtol=0, atol=0)
    if slot:
        # both gradients live in the flat buffer (no copy into it by a hook)
        assert wa.grad.data_ptr() == flat.data_ptr() and va.grad.data_ptr() == flat.data_ptr() + 8 * 4
        torch.testing.assert_close(flat[:8], wb.grad, rtol=1e-6, atol=1e-6)
    # the hook saw w's final gradient exactly once (autograd's own calls with no gradient aside)
    seen = [g for is_w, g in calls if is_w and g is not None]
    assert len(seen) == 1
    torch.testing.assert_close(seen[0], wb.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('slot', [False, True])
def test_deferred_sum_accumulates_into_existing_grad(slot):
    wa, _, _, _ = _run(2, True, slot, accumulate=True)
    wb, _, _, _ = _run(2, False, slot, accumulate=True)
    torch.testing.assert_close(wa.grad, wb.grad, rtol=1e-6, atol=1e-6)


def test_multi_use_counts_reset_per_step():
    w = torch.nn.Parameter(torch.randn(3))
    grads.begin_step()
    g1 = grads.note_use(w)
    grads.note_use(w)
    assert grads.multi_use(w, g1) and not grads.single_use(w, g1)
    grads.begin_step()
    g2 = grads.note_use(w)
    assert grads.single_use(w, g2) and not grads.multi_use(w, g2)


def test_frozen_parameter_gets_no_gradient():
    """A parameter that does not require grad, used twice, is never given a .grad."""
    w = torch.nn.Parameter(torch.randn(4), requires_grad=False)
    x = torch.randn(3, 4, requires_grad=True)
    grads.begin_step()
    (_Scale.apply(x, w).sum() + _Scale.apply(x, w).sum()).backward()
    assert w.grad is None and x.grad is not None


def _step(w, xs):
    """One 'training step' as TrainStep runs it: begin_step, forward, backward, end_step."""
    grads.begin_step()
    try:
        loss = sum((_Scale.apply(x, w) ** 2).sum() for x in xs)
        loss.backward()
    finally:
        grads.end_step()


def test_autograd_grad_after_a_step():
    """After a step, an eager forward using w twice outside any step must not defer: the
    gradient comes back from torch.autograd.grad and w.grad is left alone."""
    torch.manual_seed(1)
    w = torch.nn.Parameter(torch.randn(5))
    xs = [torch.randn(3, 5) for _ in range(2)]
    _step(w, xs)
    w.grad = None
    loss = sum((_Scale.apply(x, w) ** 2).sum() for x in xs)
    (g,) = torch.autograd.grad(loss, [w])
    w2 = torch.nn.Parameter(w.detach().clone())
    ref = sum(((x * w2) ** 2).sum() for x in xs)
    (gr,) = torch.autograd.grad(ref, [w2])
    torch.testing.assert_close(g, gr, rtol=1e-6, atol=1e-6)
    assert w.grad is None


def test_eager_use_after_a_step_matches_autograd():
    torch.manual_seed(2)
    w = torch.nn.Parameter(torch.randn(5))
    xs = [torch.randn(3, 5) for _ in range(3)]
    _step(w, xs)
    w.grad = None
    (sum((_Scale.apply(x, w) ** 2).sum() for x in xs)).backward()
    w2 = torch.nn.Parameter(w.detach().clone())
    (sum(((x * w2) ** 2).sum() for x in xs)).backward()
    torch.testing.assert_close(w.grad, w2.grad, rtol=1e-6, atol=1e-6)


def test_multi_use_non_leaf_weight_reaches_its_leaf():
    """A non-leaf weight (a DataParallel replica's, a cast copy) used twice in a step: its
    gradient must flow back to the leaf, not be parked in the non-leaf's .grad."""
    torch.manual_seed(3)
    leaf = torch.nn.Parameter(torch.randn(6))
    xs = [torch.randn(4, 6) for _ in range(2)]
    grads.begin_step()
    try:
        w = leaf * 1.0
        (sum((_Scale.apply(x, w) ** 2).sum() for x in xs)).backward()
    finally:
        grads.end_step()
    leaf2 = torch.nn.Parameter(leaf.detach().clone())
    (sum(((x * leaf2) ** 2).sum() for x in xs)).backward()
    torch.testing.assert_close(leaf.grad, leaf2.grad, rtol=1e-6, atol=1e-6)
