"""Device-side timeline probes (diagnostics; tools/step_timeline.py).  With EWVIT_PROBE=1 the
step records the device wall clock when each stream reaches a marked point: stamp(i) in the
forward, tap(x, i) at the point x's gradient arrives in the backward (an identity autograd node
whose backward stamps on the stream autograd replays it on).  Off (the default) both are
no-ops, so the step's graph carries no probe nodes."""
import os

import torch

from . import _lib as L

ON = os.environ.get('EWVIT_PROBE', '0') == '1'
NSLOT = 64
_buf = {}


def buffer(device):
    b = _buf.get(device)
    if b is None:
        b = _buf[device] = torch.zeros(NSLOT, dtype=torch.int64, device=device)
    return b


def stamp(i, device):
    if ON:
        L.call('ewvit_probe', L.ptr(buffer(device)), int(i), L.stream(buffer(device)))


class _Tap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, i):
        ctx.i = i
        ctx.dev = x.device
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        stamp(ctx.i, ctx.dev)
        return g, None


def tap(x, i):
    return _Tap.apply(x, i) if ON and x.requires_grad else x


def read(device):
    """{slot: milliseconds since slot 0} of the stamps recorded so far."""
    khz = int(L.load().ewvit_wall_clock_khz()) or 100000
    v = buffer(device).cpu().tolist()
    return {i: (t - v[0]) / khz for i, t in enumerate(v) if t}
