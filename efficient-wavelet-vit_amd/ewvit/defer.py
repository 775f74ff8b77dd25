"""Deferred weight-gradient reductions (csrc/reduce_jobs.h, include/ewvit.h).

The backbone's split-K weight gradients (1x1 expand / project convs, the FusedMBConv 3x3
convs) and its fused depthwise backward end with a small reduce launch over fp32 partial
slabs: ~110 kernel boundaries of ~5 us per backbone backward, all on the critical path.
When nothing reads the gradient before the end of the backward pass, the op marks its call
"defer": the library queues the reduce on the stream, the next weight-gradient launch on
that stream runs it in extra workgroups ahead of its own tiles, and ``flush()`` launches what
is left.  Same reduce code and summation order: bit-identical gradients.

Safe only when the gradient tensor is not read before ``flush()``: ops defer only when
they write a parameter's gradient slot (``ewvit.grads``: AccumulateGrad adopts the tensor
without reading it).  The readers flush first: the end of the backward pass (an engine
callback queued by the first deferral), ``grads._settle`` (multi-use sums), and the
data-parallel bucket all-reduce (``graph.GradBuckets._fire``).  The partial slabs stay
allocated until ``flush()``, and so do the dW tensors (a backward pass that raises before
its end leaves jobs that the next deferral flushes into them).  ``EWVIT_DEFER_REDUCE=0``
turns the deferral off (A/B).

Replaces nothing in the reference: torch's weight-gradient convs inside the backbone
(network/sfe.py:111-113) reduce internally.
"""
import ctypes
import os
import threading

import torch

from . import _lib as L

ENABLED = os.environ.get('EWVIT_DEFER_REDUCE', '1') != '0'

_lock = threading.Lock()
_held = {}            # stream handle -> (stream, [workspaces kept alive until the flush])
_queued = -1          # graph task whose end-of-backward flush is queued (the engine may run it on any thread)


def available():
    return ENABLED and hasattr(L.load(), 'ewvit_reduce_defer_next')


def mark(ws, out, device):
    """Make the next reduce-producing library call on this thread defer its reduce, keeping
    `ws` (its partial-slab workspace) and the memory of `out` (the dW it writes) alive until
    ``flush()``.
    Call right before the call.  False (nothing marked) outside a backward pass, where no
    flush would follow."""
    global _queued
    task = torch._C._current_graph_task_id()
    if task < 0:
        return False
    stale = False
    with _lock:
        if _queued != task:
            # another graph task: a nested backward (its end flushes everything, which is safe) or
            # one that raised before its end — its jobs run now, into tensors kept alive here
            stale = _queued >= 0 and bool(_held)
            try:
                torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
            except RuntimeError:
                return False
            _queued = task
    if stale:
        flush()
    with _lock:
        st = torch.cuda.current_stream(device)
        # (dW's storage, not the tensor: another reference to the tensor object would make
        # AccumulateGrad clone — read — it instead of adopting it)
        _held.setdefault(st.cuda_stream, (st, []))[1].extend((ws, out.untyped_storage()))
    L.load().ewvit_reduce_defer_next(1)
    return True


def _end_of_backward():
    global _queued
    with _lock:
        _queued = -1
    flush()


def flush():
    """Launch every deferred reduce on its stream (the current stream then waits for those
    streams) and release the kept workspaces (stream-ordered after the reduces)."""
    with _lock:
        ents = list(_held.values())
        _held.clear()
    if not ents:
        return
    lib = L.load()
    for st, _ in ents:
        rc = lib.ewvit_reduce_flush(ctypes.c_void_p(st.cuda_stream))
        if rc != 0:
            raise RuntimeError(f'ewvit_reduce_flush failed (rc={rc}): {lib.ewvit_last_error().decode()}')
    cur = torch.cuda.current_stream(ents[0][0].device)
    for st, _ in ents:
        if st != cur:
            cur.wait_stream(st)


def pending():
    """Jobs queued in the library (all streams)."""
    return int(L.load().ewvit_reduce_pending(None)) if available() else 0
