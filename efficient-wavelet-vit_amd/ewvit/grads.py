"""Gradient slots: parameter gradients written straight into a data-parallel flat buffer;
and the weight-gradient stream.

``ewvit.graph.GradBuckets`` lays every trainable parameter's gradient out in ONE flat
fp32 buffer (bucket-contiguous, in the order backward produces them) and tags each
parameter with its place there (``param._ewvit_grad_slot`` = (buffer, offset)).  A
backward kernel that produces a weight gradient asks ``grad_out`` for its output: while
the parameter holds no gradient yet it gets a FRESH view of its slot (the parameter's own
shape and strides), so the wgrad kernel writes into the all-reduce buffer itself and
autograd's AccumulateGrad adopts that view as ``param.grad`` — it steals an incoming
gradient only when nothing else references the tensor object and its layout matches, so
the view is built per call rather than kept — no clone, no copy back.
When the parameter already holds a gradient (gradient accumulation over micro-batches) a
fresh tensor is returned and AccumulateGrad adds it as usual.  The uses are counted per
step: ``begin_step`` opens a step, the ops' forwards call ``note_use``.

A parameter used more than once in the step (DAMA's frame chunks run every weight once per
chunk, dama.py:179-186) would have autograd sum its uses' gradients — one add launch per
parameter per extra use, ~560 small launches per step at config 5 — and AccumulateGrad copy
the sum into the slot.  Instead the ops hand each use's gradient to ``give``, which keeps it
and returns None to autograd; the first use in backward order writes straight into the slot
(``grad_out``), and one callback at the end of the backward pass sums every kept gradient with
``torch._foreach_add_`` (a few multi-tensor launches for all parameters), sets ``param.grad``
and runs the parameter's post-accumulate hooks (the data-parallel buckets).

Use counts are per thread: nn.DataParallel runs its replicas' forwards in threads
(reference train.py:249-251), each with its own parameters.

(A second stream for the weight gradients was built and measured slower — 2958 vs 2956
frames/s deferring nothing, 2268-2281 deferring the small wgrads, DESIGN §5.5 — and removed.)
"""
import itertools
import threading

import torch

_tls = threading.local()
_steps = itertools.count(1)     # step ids unique across threads


def begin_step():
    """A new forward (of the calling thread): use counts restart."""
    _tls.gen = next(_steps)


def end_step():
    """Close the calling thread's step (after its backward): later forwards outside a step
    (eager evaluation, a plain training loop) count no uses, so no parameter of theirs looks
    multi-use and ``give`` hands every gradient straight back to autograd."""
    _tls.gen = 0


def _gen():
    return getattr(_tls, 'gen', 0)


def note_use(param):
    """Count one use of `param` in the calling thread's current step; returns the step id,
    which the op keeps for its backward (autograd runs backward nodes on its own device
    threads, so the backward cannot read the forward thread's step)."""
    g = _gen()
    if param is None:
        return g
    if getattr(param, '_ewvit_gen', None) != g:
        param._ewvit_gen = g
        param._ewvit_uses = 1
    else:
        param._ewvit_uses += 1
    return g


def single_use(param, gen=None):
    """True when `param` entered step `gen`'s forward (default: the calling thread's current
    step) exactly once (never noted: False — unknown use counts take the conservative path)."""
    g = _gen() if gen is None else gen
    return g != 0 and getattr(param, '_ewvit_gen', None) == g and param._ewvit_uses == 1


def multi_use(param, gen):
    """True when `param` entered step `gen`'s forward more than once."""
    return (gen is not None and gen != 0 and getattr(param, '_ewvit_gen', None) == gen and
            getattr(param, '_ewvit_uses', 0) > 1)


def _slot_view(param, dtype=torch.float32):
    slot = getattr(param, '_ewvit_grad_slot', None)
    if slot is not None and param.is_leaf and param.grad is None and slot[0].dtype == dtype:
        return slot[0].as_strided(param.shape, param.stride(), slot[1])
    return None


def is_slot(param, t):
    """True when `t` is `param`'s gradient slot (what ``grad_out`` hands out for it): a tensor
    AccumulateGrad adopts, or ``give`` keeps for the end-of-backward sum, without reading it."""
    view = _slot_view(param, t.dtype)
    return view is not None and view.data_ptr() == t.data_ptr() and view.stride() == t.stride()


def deferrable(param, t, gen):
    """True when nothing reads `t` — the gradient of `param` an op's backward is about to write
    — before the end of the backward pass, so its last kernel may be deferred (ewvit.defer):
    the gradient slot (AccumulateGrad adopts it; the data-parallel hook and the multi-use sum
    flush first), a multi-use parameter's gradient (``give`` keeps it for the end-of-backward
    sum, which flushes first), or a fresh tensor of a single-use leaf with no gradient and no
    hooks (AccumulateGrad steals it: default layout, no other reference)."""
    if param is None or not param.is_leaf or not param.requires_grad:
        return False
    if torch.is_grad_enabled():
        # a create_graph backward: AccumulateGrad clones (reads) the gradient instead of adopting it
        return False
    if getattr(param, '_ewvit_early', False):        # updated as soon as its gradient lands (TrainStep)
        return False
    if is_slot(param, t):
        return True
    if param.grad is not None or getattr(param, '_backward_hooks', None) or \
            getattr(param, '_post_accumulate_grad_hooks', None):
        return False
    if DEFER and multi_use(param, gen):
        return True
    return single_use(param, gen) and t.is_contiguous(memory_format=torch.contiguous_format) == \
        param.is_contiguous(memory_format=torch.contiguous_format) and t.stride() == param.stride()


def grad_out(param, gen=None, dtype=torch.float32):
    """Output tensor for `param`'s gradient (shape and strides of `param`); `gen`: the step id
    `note_use` returned in the op's forward.  The slot itself for a single use, and for the
    first use in backward order of a parameter used several times (``give`` defers the sum)."""
    view = _slot_view(param, dtype)
    if view is not None:
        if single_use(param, gen):
            return view
        if DEFER and multi_use(param, gen) and getattr(param, '_ewvit_slot_gen', None) != gen:
            param._ewvit_slot_gen = gen
            return view
    return torch.empty_like(param, dtype=dtype, memory_format=torch.preserve_format)


# ---- deferred sums of multi-use parameters' gradients
DEFER = True            # False: autograd sums the uses (the test switch, tests/test_gpu_grads.py)
_lock = threading.Lock()
_pending = {}           # step id -> {id(param): [param, [gradients], {streams}]}
_queued = set()


def give(param, g, gen):
    """What an op's backward returns to autograd for `param`'s gradient `g`: `g` itself, or —
    for a parameter used more than once in step `gen` — None, with `g` kept for the sum at the
    end of the backward pass."""
    # (only a leaf is deferred: the sum is written to param.grad, which autograd would never
    # propagate from a non-leaf weight — a DataParallel replica's, a cast copy — to its leaf)
    if (g is None or param is None or not DEFER or not param.requires_grad or not param.is_leaf
            or not multi_use(param, gen)):
        return g
    with _lock:
        ent = _pending.setdefault(gen, {}).setdefault(id(param), [param, [], set()])
        ent[1].append(g)
        if g.is_cuda:
            ent[2].add(torch.cuda.current_stream(g.device))
        first = gen not in _queued
        _queued.add(gen)
    if first:
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _settle(gen))
    return None


def _settle(gen):
    """End of the backward pass: every kept gradient summed into its parameter's gradient."""
    with _lock:
        ents = list(_pending.pop(gen, {}).values())
        _queued.discard(gen)
    if not ents:
        return
    from . import defer
    defer.flush()                     # deferred weight-gradient reductions land first
    cuda = [e for e in ents if e[1][0].is_cuda]
    if cuda:
        cur = torch.cuda.current_stream(cuda[0][1][0].device)
        seen = set()
        for _, _, streams in cuda:
            for st in streams:
                if st != cur and st not in seen:
                    seen.add(st)
                    cur.wait_stream(st)
    copy_dst, copy_src, rounds, finals = [], [], [], []
    for p, ts, _ in ents:
        rest = ts
        if p.grad is not None:                       # accumulation over micro-batches
            base = p.grad
        else:
            view = _slot_view(p)
            hit = None if view is None else next((i for i, t in enumerate(ts) if t.data_ptr() == view.data_ptr()), None)
            if hit is not None:                      # the first use wrote into the slot
                base, rest = ts[hit], ts[:hit] + ts[hit + 1:]
            elif view is not None:
                base, rest = view, ts[1:]
                copy_dst.append(view)
                copy_src.append(ts[0])
            else:
                base, rest = ts[0], ts[1:]
        finals.append((p, base))
        for k, t in enumerate(rest):
            if len(rounds) <= k:
                rounds.append(([], []))
            rounds[k][0].append(base)
            rounds[k][1].append(t)
    if copy_dst:
        torch._foreach_copy_(copy_dst, copy_src)
    for dst, src in rounds:
        torch._foreach_add_(dst, src)
    for p, base in finals:
        if p.grad is None:
            p.grad = base
        hooks = getattr(p, '_post_accumulate_grad_hooks', None)
        for h in (list(hooks.values()) if hooks else []):
            h(p)


def set_slot(param, flat, offset):
    """`param`'s gradient lives at `flat[offset:]` with the parameter's own strides."""
    param._ewvit_grad_slot = (flat, offset)


def clear_slot(param):
    if hasattr(param, '_ewvit_grad_slot'):
        del param._ewvit_grad_slot
