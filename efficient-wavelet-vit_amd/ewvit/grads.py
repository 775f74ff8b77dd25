"""Gradient slots: parameter gradients written straight into a data-parallel flat buffer.

``ewvit.graph.GradBuckets`` lays every trainable parameter's gradient out in ONE flat
fp32 buffer (bucket-contiguous, in the order backward produces them) and tags each
parameter with its view (``param._ewvit_grad_slot``, the parameter's own shape and
strides).  A backward kernel that produces a weight gradient asks ``grad_out`` for its
output: while the parameter holds no gradient yet it gets the slot, so the wgrad kernel
writes into the all-reduce buffer itself and autograd's AccumulateGrad adopts that
tensor as ``param.grad`` (it steals a lone, layout-matching incoming gradient) — no copy.
When the parameter already holds a gradient (a weight used twice, gradient accumulation
over micro-batches) a fresh tensor is returned and AccumulateGrad adds it as usual.
"""
import torch


def grad_out(param, dtype=torch.float32):
    """Output tensor for `param`'s gradient (shape and strides of `param`)."""
    slot = getattr(param, '_ewvit_grad_slot', None)
    if slot is not None and param.grad is None and slot.dtype == dtype:
        return slot
    return torch.empty_like(param, dtype=dtype, memory_format=torch.preserve_format)


def set_slot(param, view):
    param._ewvit_grad_slot = view


def clear_slot(param):
    if hasattr(param, '_ewvit_grad_slot'):
        del param._ewvit_grad_slot
