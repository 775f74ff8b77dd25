"""Adam on the ewvit multi-tensor kernel (csrc/optim.hip) — the optimizer of the
reference's training step (train.py:273-275: ``optim.Adam(params, lr, weight_decay)``).

Same constructor, update rule and state layout as ``torch.optim.Adam`` (per-parameter
state ``step`` / ``exp_avg`` / ``exp_avg_sq``, so checkpoints load either way), for
amsgrad=False / maximize=False.  ``step()`` issues ONE launch per parameter group from a
device table of the tensors' addresses (rebuilt when they change; a graph capture's table is
allocated before it and filled after it, ``finish_capture()``), or — with EWVIT_ADAM_TABLE=0
or no such table — one launch per 48 tensors with the pointers passed by value; plus one foreach increment of
the per-parameter device step counters.

The learning rate is read by the kernel from a per-group device scalar (``self._lr_dev``),
written from ``group['lr']`` by ``sync_hyper()`` — called by every eager ``step()`` and, for
a step recorded in a HIP graph, by ``ewvit.graph.TrainStep`` before each replay — so an LR
scheduler (train.py:274,300: CosineAnnealingLR) drives a replayed step too.  betas, eps and
weight_decay are launch constants: ``hyper_signature()`` lets a graph owner detect a change.
"""
import ctypes

import torch

from . import _lib as L


def _dense(t):
    """True when t's elements fill exactly numel() consecutive slots (any dim order)."""
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False,
                 maximize=False, **_ignored):
        if amsgrad or maximize:
            raise NotImplementedError('ewvit.optim.Adam: amsgrad / maximize are not used by the reference')
        if lr < 0 or eps < 0 or not 0 <= betas[0] < 1 or not 0 <= betas[1] < 1 or weight_decay < 0:
            raise ValueError('ewvit.optim.Adam: invalid hyper-parameters')
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        import os
        self.table = os.environ.get('EWVIT_ADAM_TABLE', '1') != '0'   # one launch per group

    def sync_hyper(self):
        """Write each group's current lr into its device scalar (outside any graph capture).

        The scalars are keyed by group INDEX and refilled in place: ``load_state_dict``
        replaces every param_group dict, and a graph captured before it keeps reading the
        tensor it was recorded with."""
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError('ewvit.optim.Adam.sync_hyper: called inside a graph capture (the fill '
                               'would be recorded and override the schedule on every replay)')
        lrs = self.__dict__.setdefault('_lr_dev', {})      # group index -> [device f64 scalar, value]
        for gi, group in enumerate(self.param_groups):
            lr = float(group['lr'])
            dev = next((p.device for p in group['params'] if p.is_cuda), None)
            if dev is None:
                continue
            e = lrs.get(gi)
            if e is None or e[0].device != dev:
                e = lrs[gi] = [torch.empty((), dtype=torch.float64, device=dev), None]
            if e[1] != lr:
                e[0].fill_(lr)
                e[1] = lr

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict, keeping the device tensors a captured step
        reads: the loaded ``step`` / ``exp_avg`` / ``exp_avg_sq`` are copied INTO the existing
        state tensors (torch would replace them, and a HIP graph recorded before the load would
        keep updating the old ones), and the lr scalars stay keyed by group index."""
        old = {p: dict(st) for p, st in self.state.items()}
        prev_state, prev_groups = self.state, self.param_groups
        super().load_state_dict(state_dict)
        # a parameter a captured step updates must keep its tensors, else the graph would go on
        # updating the old ones while the optimizer shows the loaded, never-updated ones
        captured = self.__dict__.get('_captured_params', ())
        bad = [i for i, p in enumerate(captured)
               if not all(k in old.get(p, {}) and torch.is_tensor(self.state.get(p, {}).get(k))
                          and old[p][k].shape == self.state[p][k].shape for k in ('step', 'exp_avg', 'exp_avg_sq'))]
        if bad:
            self.__setstate__({'state': prev_state, 'param_groups': prev_groups})
            raise RuntimeError(f'ewvit.optim.Adam.load_state_dict: {len(bad)} parameter(s) a captured step updates '
                               'have no matching state in the loaded dict; re-capture the step (build a new '
                               'TrainStep) after loading such a state')
        for p, st in self.state.items():
            o = old.get(p)
            if not o:
                continue
            for k in ('step', 'exp_avg', 'exp_avg_sq'):
                if k in o and k in st and torch.is_tensor(st[k]) and o[k].shape == st[k].shape:
                    o[k].copy_(st[k])
                    st[k] = o[k]

    def hyper_signature(self):
        """The hyper-parameters a recorded step bakes in as launch constants."""
        return tuple((tuple(g['betas']), float(g['eps']), float(g['weight_decay'])) for g in self.param_groups)

    def _group_step(self, gi, group, subset=None, tag=None):
        items = []
        for p in group['params']:
            if p.grad is None or (subset is not None and id(p) not in subset):
                continue
            if p.grad.is_sparse:
                raise RuntimeError('ewvit.optim.Adam: sparse gradients are not supported')
            if p.dtype != torch.float32 or not p.is_cuda:
                raise RuntimeError('ewvit.optim.Adam: fp32 parameters on the GPU only')
            if not _dense(p):
                raise RuntimeError('ewvit.optim.Adam: parameters must be dense (no gaps or overlap)')
            st = self.state[p]
            if not st:
                st['step'] = torch.zeros((), dtype=torch.float32, device=p.device)
                st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
            elif st['step'].device != p.device:          # a loaded torch checkpoint keeps it on the host
                st['step'] = st['step'].to(device=p.device, dtype=torch.float32)
            g = p.grad
            if g.stride() != p.stride():
                g = torch.empty_like(p).copy_(g)          # same element order as p / m / v
            items.append((p, g, st))
        if not items:
            return
        torch._foreach_add_([c[2]['step'] for c in items], 1.0)   # torch semantics: per-parameter steps
        b1, b2 = group['betas']
        if gi not in self.__dict__.get('_lr_dev', {}):
            self.sync_hyper()           # raises inside a capture: never record the scalar's fill
        lr_dev = L.ptr(self._lr_dev[gi][0])
        stream = L.stream(items[0][0])
        if self._table_step(gi if tag is None else (gi, tag), group, items, lr_dev, stream):
            return
        for k in range(0, len(items), L.ADAM_MAX):
            chunk = items[k:k + L.ADAM_MAX]
            n = len(chunk)
            cols = ([c[0] for c in chunk], [c[1] for c in chunk], [c[2]['exp_avg'] for c in chunk],
                    [c[2]['exp_avg_sq'] for c in chunk], [c[2]['step'] for c in chunk])
            ptrs = [(ctypes.c_void_p * n)(*[t.data_ptr() for t in col]) for col in cols]
            numel = (ctypes.c_int64 * n)(*[c[0].numel() for c in chunk])
            L.call('ewvit_adam_step', n, ptrs[0], ptrs[1], ptrs[2], ptrs[3], numel, ptrs[4],
                   float(group['lr']), lr_dev, float(b1), float(b2), float(group['eps']),
                   float(group['weight_decay']), stream, work={'bytes': 28.0 * sum(c[0].numel() for c in chunk)})

    def _table_step(self, gi, group, items, lr_dev, stream):
        """The whole group in one launch (ewvit_adam_step_table) from a device table of its
        tensors' addresses, rebuilt when they change.

        Eager: one device table per group, refilled in place from a pinned host buffer
        (stream-ordered after the launches that read it) while its row count holds.  Capture:
        the launch reads a spare table allocated by the eager step before it (outside the
        graph's pool, so no captured temporary can alias it), filled by finish_capture() and
        owned by the graph from then on (finish_capture(graph) ties it to the graph's
        lifetime).  Without a spare, the per-48-tensor launches above.  EWVIT_ADAM_TABLE=0: off."""
        if not self.table:
            return False
        key = tuple((c[0].data_ptr(), c[1].data_ptr(), c[2]['exp_avg'].data_ptr(), c[2]['exp_avg_sq'].data_ptr(),
                     c[2]['step'].data_ptr(), c[0].numel()) for c in items)
        tables = self.__dict__.setdefault('_tables', {})   # gi -> [key, device table, chunks, graph-owned]
        spares = self.__dict__.setdefault('_spare', {})
        capturing = torch.cuda.is_current_stream_capturing()
        cached = tables.get(gi)
        if cached is None or cached[0] != key:
            lib, rows, chunk0 = L.load(), [], 0
            for k in key:
                rows.append(list(k) + [chunk0])
                chunk0 += int(lib.ewvit_adam_chunks(k[5]))
            if capturing:
                tab = spares.pop(gi, None)
                if tab is None or tab.shape[0] != len(rows):
                    return False
                self.__dict__.setdefault('_fill_after_capture', []).append((tab, rows))
                cached = tables[gi] = [key, tab, chunk0, True]
            else:
                dev = items[0][0].device
                if cached is not None and not cached[3] and cached[1].shape[0] == len(rows):
                    tab = cached[1]                     # refill in place (same stream as its readers)
                else:
                    tab = torch.empty((len(rows), 7), dtype=torch.int64, device=dev)
                pin = self.__dict__.get('_pin', {}).get(gi)
                if pin is None or pin[0].shape[0] != len(rows):
                    pin = self.__dict__.setdefault('_pin', {})[gi] = [
                        torch.empty((len(rows), 7), dtype=torch.int64, pin_memory=True), None]
                if pin[1] is not None:
                    pin[1].synchronize()               # the previous copy out of it has finished
                pin[0].copy_(torch.tensor(rows, dtype=torch.int64))
                tab.copy_(pin[0], non_blocking=True)
                pin[1] = torch.cuda.Event()
                pin[1].record()
                if spares.get(gi) is None or spares[gi].shape[0] != len(rows):
                    spares[gi] = torch.empty_like(tab)
                cached = tables[gi] = [key, tab, chunk0, False]
        elif capturing and not cached[3]:
            # the same addresses as the eager table: the graph must not share a table an
            # eager rebuild may refill, so it takes the spare with the same rows
            tab = spares.pop(gi, None)
            if tab is None or tab.shape != cached[1].shape:
                return False
            self.__dict__.setdefault('_fill_after_capture', []).append((tab, None, cached[1]))
            cached = tables[gi] = [key, tab, cached[2], True]
        b1, b2 = group['betas']
        L.call('ewvit_adam_step_table', L.ptr(cached[1]), len(key), cached[2], float(group['lr']), lr_dev, float(b1),
               float(b2), float(group['eps']), float(group['weight_decay']), stream,
               work={'bytes': 28.0 * sum(k[5] for k in key)})
        return True

    def finish_capture(self, graph=None):
        """Fill the tables a graph capture launched Adam on (their rows are host data; the
        replays only read them) and hand them to the graph: with ``graph`` given they live as
        long as it does (ewvit.graph.TrainStep passes its graphs), else the optimizer keeps
        them.  Returns the tables."""
        out = []
        cap = self.__dict__.setdefault('_captured_params', [])
        have = set(map(id, cap))
        cap.extend(p for p, st in self.state.items() if st and id(p) not in have)
        for item in self.__dict__.pop('_fill_after_capture', []):
            tab = item[0]
            if item[1] is not None:
                tab.copy_(torch.tensor(item[1], dtype=torch.int64))
            else:
                tab.copy_(item[2])
            out.append(tab)
        if graph is not None:
            graph.__dict__.setdefault('_ewvit_adam_tables', []).extend(out)
        else:
            self.__dict__.setdefault('_table_keep', []).extend(out)
        return out

    def release_capture(self):
        """The graphs that launched Adam on this optimizer's state were released
        (``ewvit.graph.TrainStep.close``): forget which parameters a captured step updates —
        ``load_state_dict`` stops insisting on their state — and drop the tables kept here."""
        self.__dict__.pop('_captured_params', None)
        self.__dict__.pop('_table_keep', None)
        self.__dict__.pop('_fill_after_capture', None)

    def launches_per_step(self):
        """Adam kernel launches one step makes, by kernel name, in either launch form (the
        profilers count step equivalents from them, whichever form the profiled build took)."""
        groups = [sum(1 for p in g['params'] if p.requires_grad) for g in self.param_groups]
        k = int(self.__dict__.get('_split_steps', 1))      # step_subset calls per step (TrainStep early_params)
        return {'adam_table_kernel': k * sum(1 for n in groups if n),
                'adam_multi_kernel': sum(-(-n // L.ADAM_MAX) for n in groups) + (k - 1) * sum(1 for n in groups if n)}

    @torch.no_grad()
    def step_subset(self, tag, params):
        """``step()`` restricted to `params` (a set of parameter ids): the same per-parameter
        update, launched on the current stream with its own device table (`tag` names it).  The
        training step uses it to update the parameters whose gradients are final before the end of
        the backward pass early, on a side stream (ewvit.graph.TrainStep ``early_params``)."""
        if not torch.cuda.is_current_stream_capturing():
            self.sync_hyper()
        for gi, group in enumerate(self.param_groups):
            self._group_step(gi, group, params, tag)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not torch.cuda.is_current_stream_capturing():
            self.sync_hyper()           # a captured step reads the scalar its owner refreshes
        for gi, group in enumerate(self.param_groups):
            self._group_step(gi, group)
        return loss
