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
When the parameter already holds a gradient (gradient accumulation over micro-batches) or
is used more than once in the step (DAMA's frame chunks run every weight once per chunk:
autograd sums the uses' gradients before AccumulateGrad, so two uses must not share one
slot) a fresh tensor is returned and AccumulateGrad adds it as usual.  The uses are
counted per step: ``begin_step`` opens a step, the ops' forwards call ``note_use``.

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


def grad_out(param, gen=None, dtype=torch.float32):
    """Output tensor for `param`'s gradient (shape and strides of `param`); `gen`: the step id
    `note_use` returned in the op's forward."""
    slot = getattr(param, '_ewvit_grad_slot', None)
    if slot is not None and param.is_leaf and param.grad is None and slot[0].dtype == dtype and single_use(param, gen):
        return slot[0].as_strided(param.shape, param.stride(), slot[1])
    return torch.empty_like(param, dtype=dtype, memory_format=torch.preserve_format)


def set_slot(param, flat, offset):
    """`param`'s gradient lives at `flat[offset:]` with the parameter's own strides."""
    param._ewvit_grad_slot = (flat, offset)


def clear_slot(param):
    if hasattr(param, '_ewvit_grad_slot'):
        del param._ewvit_grad_slot
