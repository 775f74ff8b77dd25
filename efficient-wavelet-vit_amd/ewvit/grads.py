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

**Weight-gradient stream.**  A weight gradient is off the backward's critical path: only
the optimizer (and the data-parallel all-reduce) reads it, while the input gradient feeds
the next layer's backward.  With ``set_wgrad_stream(True)`` (``ewvit.graph.TrainStep``
with ``EWVIT_WGRAD_STREAM=1``) a conv whose weight is used once in the step issues its
wgrad (if at least ``EWVIT_WGRAD_MIN_FLOPS``) on a second stream, to fill the CUs the
latency-bound input-gradient chain leaves idle.  The stream waits for the main stream at
the point of issue (dy and x are ready), the tensors it reads are recorded on it (the
caching allocator keeps them until it is done), and every consumer joins it: the bucket
all-reduces (``wgrad_wait``), any synchronous gradient of a parameter that might already
hold a deferred one (``wgrad_wait``), and the end of each backward (``wgrad_join``), which
also rejoins the stream before a HIP-graph capture ends.  OFF by default: measured on the
config-2 step it loses — 2958 vs 2956 frames/s deferring nothing (threshold 1e12), 2901 at
5e9 FLOPs, 2268-2281 at 2e9 and below: the concurrent wgrads lengthen the
dgrad chain more than they save.
"""
import os

import torch

DEFER_MIN_FLOPS = float(os.environ.get('EWVIT_WGRAD_MIN_FLOPS', '0'))
_gen = 0
_enabled = False
_streams = {}
_issued = set()          # devices with wgrad work issued since the last join


def begin_step():
    """A new forward: use counts restart."""
    global _gen
    _gen += 1


def note_use(param):
    if param is None:
        return
    if getattr(param, '_ewvit_gen', None) != _gen:
        param._ewvit_gen = _gen
        param._ewvit_uses = 1
    else:
        param._ewvit_uses += 1


def single_use(param):
    """True when `param` entered the current step's forward exactly once (never noted:
    False — unknown use counts take the conservative path)."""
    return getattr(param, '_ewvit_gen', None) == _gen and param._ewvit_uses == 1


def grad_out(param, dtype=torch.float32):
    """Output tensor for `param`'s gradient (shape and strides of `param`)."""
    slot = getattr(param, '_ewvit_grad_slot', None)
    if slot is not None and param.is_leaf and param.grad is None and slot[0].dtype == dtype and single_use(param):
        return slot[0].as_strided(param.shape, param.stride(), slot[1])
    return torch.empty_like(param, dtype=dtype, memory_format=torch.preserve_format)


def set_slot(param, flat, offset):
    """`param`'s gradient lives at `flat[offset:]` with the parameter's own strides."""
    param._ewvit_grad_slot = (flat, offset)


def clear_slot(param):
    if hasattr(param, '_ewvit_grad_slot'):
        del param._ewvit_grad_slot


# ---------------------------------------------------------------- weight-gradient stream
def set_wgrad_stream(on):
    global _enabled
    prev, _enabled = _enabled, bool(on)
    return prev


def wgrad_stream(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _streams.get(idx)
    if st is None:
        st = _streams[idx] = torch.cuda.Stream(device=torch.device('cuda', idx))
    return st


def deferrable(*params):
    """The weight gradient of these parameters may go to the wgrad stream: the stream is
    on, and each parameter (None = no gradient wanted) holds no gradient and was used once
    — so AccumulateGrad adopts the deferred tensor without a kernel of its own on the
    main stream (the op's output must keep the parameter's layout for that)."""
    if not _enabled:
        return False
    return all(p is None or (p.is_leaf and p.grad is None and single_use(p)) for p in params)


def defer_begin(device, *reads):
    """Fork: the wgrad stream waits for the current stream; `reads` (dy, x, …) are kept
    alive for it.  Returns the stream (use it as the current stream for the launches)."""
    cur = torch.cuda.current_stream(device)
    st = wgrad_stream(device)
    st.wait_stream(cur)
    for t in reads:
        if t is not None:
            t.record_stream(st)
    _issued.add(st.device.index)
    return st


def defer_output(t, device):
    """A gradient tensor written on the wgrad stream and handed to autograd on the
    current one: its memory is in use on both."""
    t.record_stream(torch.cuda.current_stream(device))


def wgrad_wait(device):
    """The current stream waits for every wgrad issued so far (a consumer, or a synchronous
    gradient that AccumulateGrad may add to a deferred one)."""
    if device.type == 'cuda' and (device.index if device.index is not None else torch.cuda.current_device()) in _issued:
        torch.cuda.current_stream(device).wait_stream(wgrad_stream(device))


def wgrad_join():
    """End of a backward: the current stream joins the wgrad stream of every device used."""
    for idx in list(_issued):
        dev = torch.device('cuda', idx)
        torch.cuda.current_stream(dev).wait_stream(wgrad_stream(dev))
    _issued.clear()
