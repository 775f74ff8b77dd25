"""A static-shape data-parallel training step, replayed from one captured HIP graph.

The reference's training iteration (train.py:93-115: DeepfakeDetector forward over
the chunk, combined_loss, backward, optimizer step; `nn.DataParallel` at train.py:249-251
for --multi-gpu) issues ~1500 kernel launches; issued from Python each costs 10-50 us of
host time, more than the GPU needs for most of them.  `TrainStep` records the whole
iteration once into a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm) and replays it:
one host call per step.

Data parallel (one process per GPU, RCCL over xGMI) — `GradBuckets`:

* every trainable gradient lives in ONE flat fp32 buffer, laid out in the order backward
  produces the gradients (observed on the first step and agreed from rank 0, as DDP
  rebuilds its buckets) and cut into ~`bucket_mb` buckets;
* the conv / linear wgrad kernels write their gradient straight into the buffer
  (ewvit.grads slots); the few gradients autograd allocates itself are copied in by the
  parameter's post-accumulate hook;
* as soon as a bucket's last gradient lands, its all-reduce (average) is issued — in
  bucket order — on the process group's stream, so the ring over xGMI runs under the rest
  of the backward (the patch_to_embedding bucket, 128 MB, under the backbone's backward);
* the optimizer waits for the buckets and reads the gradients as views of the buffer.

With a capturable backend (RCCL) the collectives are recorded in the same graph as
forward, backward and the optimizer.  The module buffers (BatchNorm running statistics
and counters) are re-pointed into flat buffers and broadcast from rank 0 at the start of
every step — inside the graph — which is what DistributedDataParallel(broadcast_buffers=
True) does and what the reference's DataParallel replicas see (the replicas copy device
0's buffers every forward).  BN batch statistics and the `pos_embedding[0:N]` chunk
position stay per replica.  gloo (the CPU tests, the one-GPU rehearsal) runs the same
sequence eagerly.

Replay-time inputs: the optimizer's learning rate is a device scalar refreshed before each
replay (ewvit.optim.Adam.sync_hyper) so an LR scheduler keeps working; other per-step
values (e.g. the curriculum weight of combined_loss, train.py:76-86: pass `weight=` a device
tensor the caller updates in place) must be device tensors too; betas / eps / weight decay
are launch constants and a change raises.  `accum_steps=k` records k forward/backward
passes (forward_loss(micro) for micro in 0..k-1, each loss / k, train.py:110-115) before
the reduction and the optimizer step.

Requirements of graph mode: every input of `forward_loss` is a static tensor updated in
place, the model issues no host synchronisation, and random draws use the device
generator (torch ops) or the ewvit dropout step counter (_lib.rng_advance, advanced
inside the recorded forward).
"""
import os

import torch
import torch.distributed as dist

from . import grads
from .grads import clear_slot, set_slot


def _world(group):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _backend(group):
    return dist.get_backend(group) if _world(group) > 1 else None


def _pg_status():
    """The flight recorder's per-process-group status, {} when this torch build or process
    group does not provide it (private API: a missing symbol, another signature or an
    unparsable dump all read as 'unavailable', never as an exception)."""
    import json
    try:
        from torch._C import _distributed_c10d as c10d
        d = json.loads(c10d._dump_nccl_trace_json(includeCollectives=False, onlyActive=True))
        st = d.get('pg_status') if isinstance(d, dict) else None
        return st if isinstance(st, dict) else {}
    except Exception:            # noqa: BLE001 — AttributeError / TypeError / ValueError / RuntimeError
        return {}


def retire_eager_collectives(timeout_s=60.0):
    """Block until ProcessGroupNCCL's watchdog has retired every collective issued so far
    (device synchronised first).  Raises if the status is unavailable or the watchdog does
    not catch up within `timeout_s`."""
    import time
    torch.cuda.synchronize()
    t0 = time.monotonic()
    while True:
        st = _pg_status()
        if not st:
            raise RuntimeError('TrainStep: the process-group status (flight recorder pg_status) is unavailable, '
                               'so the watchdog queue cannot be drained before a global-mode capture: set '
                               'TORCH_FR_BUFFER_SIZE (e.g. 2000) before init_process_group, or use the default '
                               'EWVIT_CAPTURE_MODE=relaxed')
        behind = {k: v for k, v in st.items()
                  if int(v.get('last_completed_collective', -1)) < int(v.get('last_enqueued_collective', -1))}
        if not behind:
            return
        if time.monotonic() - t0 > timeout_s:
            raise RuntimeError(f'TrainStep: the NCCL watchdog did not retire the eager collectives: {behind}')
        time.sleep(0.005)


class GradBuckets:
    """Flat, bucketed gradient buffer with all-reduces issued as buckets fill.

    ``force=True`` issues the collectives even in a world of one process (a test switch: it
    puts the RCCL calls inside the captured step graph on a one-GPU box).

    ``comm_dtype=torch.bfloat16`` (opt-in; EWVIT_GRAD_COMM_DTYPE=bf16 for TrainStep): each
    bucket is rounded to bf16 into a communication buffer and all-reduced there — half the
    xGMI bytes of the fp32 gradient (240 MB -> 120 MB per step at config 2) — and the
    averaged result is widened back into the fp32 buffer the optimizer reads (fp32 master
    weights and Adam slots are untouched).  The gradient then carries one bf16 rounding per
    rank before the sum (a relative error of ~2^-9 per element), which the reference's fp32
    DataParallel gradient does not; default off."""

    def __init__(self, params, group=None, bucket_mb=32, first_bucket_mb=4, force=False, comm_dtype=None):
        self.params = list(params)
        self.group = group
        self.comm_dtype = comm_dtype if comm_dtype not in (None, torch.float32) else None
        if self.comm_dtype is not None and self.comm_dtype != torch.bfloat16:
            raise ValueError(f'GradBuckets: comm_dtype {comm_dtype} (float32 or bfloat16)')
        self.world = _world(group)
        self.reduce = self.world > 1 or (force and dist.is_available() and dist.is_initialized())
        self.avg_op = not self.reduce or dist.get_backend(group) != 'gloo'   # gloo has no AVG: SUM, then divide
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.first_bytes = min(int(first_bucket_mb * (1 << 20)), self.bucket_bytes)
        self.order = None          # parameter indices in gradient-ready order
        self.observed = []
        self.collect = True        # only the last micro-batch of a step reduces
        self.defer = False         # True: no collectives from the hooks (all-reduce_all() after)
        self.flat = None
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook(i)) for i, p in enumerate(self.params)]
        self._layout(list(range(len(self.params)))[::-1])      # DDP's first guess: reverse registration

    # ---- layout
    def _layout(self, order):
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        self.order = list(order)
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.comm = torch.zeros(n, dtype=self.comm_dtype, device=dev) if self.comm_dtype is not None else None
        self.views = [None] * len(self.params)
        self.bucket_of = [0] * len(self.params)
        self.buckets = []          # [(start, end, [param idx])]
        off, start, cur, cap = 0, 0, [], self.first_bytes
        for i in self.order:
            p = self.params[i]
            self.views[i] = self.flat.as_strided(p.shape, p.stride(), off)    # the parameter's own strides
            set_slot(p, self.flat, off)
            if cur and (off - start + p.numel()) * 4 > cap:
                self.buckets.append((start, off, cur))
                start, cur, cap = off, [], self.bucket_bytes
            cur.append(i)
            self.bucket_of[i] = len(self.buckets)
            off += p.numel()
        if cur:
            self.buckets.append((start, off, cur))

    def relayout(self):
        """Re-cut the buffer in the order the last backward produced the gradients
        (rank 0's order, so every rank issues the same collectives in the same order)."""
        seen = list(dict.fromkeys(self.observed))
        order = seen + [i for i in reversed(range(len(self.params))) if i not in set(seen)]
        if self.reduce:
            t = torch.tensor(order, dtype=torch.int64, device=self.flat.device)
            dist.broadcast(t, 0, group=self.group)
            order = t.tolist()
        if order != self.order:
            self._layout(order)

    # ---- one step
    def begin(self):
        self.pending = [len(b[2]) for b in self.buckets]
        self.next = 0
        self.works = []
        self.observed = []
        self.streams = [set() for _ in self.buckets]     # streams that wrote each bucket

    def _hook(self, i):
        def hook(p):
            # (a parameter whose uses all deferred their gradients to ewvit.grads' end-of-backward
            # sum reaches AccumulateGrad with none: its hook runs again once the sum is in)
            if not self.collect or p.grad is None:
                return
            self.observed.append(i)
            v = self.views[i]
            if p.grad is not v:
                if p.grad.data_ptr() != v.data_ptr():
                    v.copy_(p.grad)
                p.grad = v
            b = self.bucket_of[i]
            if v.is_cuda:
                self.streams[b].add(torch.cuda.current_stream(v.device))
            self.pending[b] -= 1
            self._fire_ready()
        return hook

    def _fire(self, b):
        s, e, _ = self.buckets[b]
        if self.reduce and not self.defer:
            if self.flat.is_cuda:
                from . import defer
                defer.flush()                # deferred weight-gradient reductions land first
                # the gradients of a bucket may come from several streams (DAMA's MWT branch
                # runs on its own): the collective, issued on the current stream, waits for all
                cur = torch.cuda.current_stream(self.flat.device)
                for st in self.streams[b]:
                    if st != cur:
                        cur.wait_stream(st)
            op = dist.ReduceOp.AVG if self.avg_op else dist.ReduceOp.SUM
            buf = self.flat[s:e]
            if self.comm is not None:
                buf = self.comm[s:e]
                buf.copy_(self.flat[s:e])            # round to the communication dtype
            self.works.append(dist.all_reduce(buf, op=op, group=self.group, async_op=True))

    def _fire_ready(self):
        while self.next < len(self.buckets) and self.pending[self.next] == 0:
            self._fire(self.next)
            self.next += 1

    def finish(self):
        """After backward: zero the slots of parameters that got no gradient, issue the
        remaining buckets, wait for all of them (a stream wait under RCCL)."""
        for b in range(self.next, len(self.buckets)):
            if self.pending[b]:
                for i in self.buckets[b][2]:
                    p = self.params[i]
                    if p.grad is None:
                        self.views[i].zero_()
                self.pending[b] = 0
        self._fire_ready()
        for w in self.works:
            w.wait()
        self.works = []
        if self.reduce and not self.defer and self.comm is not None:
            self.flat.copy_(self.comm)               # widen the reduced gradients (one launch)
        if self.reduce and not self.avg_op and not self.defer:
            self.flat.div_(self.world)

    def allreduce_all(self):
        """The deferred form: one all-reduce of the whole buffer (between two graphs)."""
        if self.reduce:
            op = dist.ReduceOp.AVG if self.avg_op else dist.ReduceOp.SUM
            if self.comm is not None:
                self.comm.copy_(self.flat)
                dist.all_reduce(self.comm, op=op, group=self.group)
                self.flat.copy_(self.comm)
            else:
                dist.all_reduce(self.flat, op=op, group=self.group)
            if not self.avg_op:
                self.flat.div_(self.world)

    def remove(self):
        for h in self._hooks:
            h.remove()
        for p in self.params:
            clear_slot(p)


class BufferSync:
    """Module buffers re-pointed into one flat tensor per dtype, broadcast from rank 0.

    Modules whose class sets ``ewvit_buffer_sync = False`` (the checkpoint placeholders of
    the reference's unused ablation heads, network/model.py) and everything below them are
    left out: nothing updates them, and they can hold hundreds of MB."""

    def __init__(self, model, group=None):
        self.group = group
        by_dt = {}
        skip = [n for n, m in model.named_modules() if getattr(type(m), 'ewvit_buffer_sync', True) is False]
        for mname, mod in model.named_modules():
            if any(mname == s or mname.startswith(s + '.') for s in skip):
                continue
            for name, b in mod._buffers.items():
                if b is not None:
                    by_dt.setdefault(b.dtype, []).append((mod, name, b))
        self.flats = []
        for dt, items in by_dt.items():
            n = sum(b.numel() for _, _, b in items)
            flat = torch.empty(n, dtype=dt, device=items[0][2].device)
            off = 0
            for mod, name, b in items:
                v = flat[off:off + b.numel()].view(b.shape)
                v.copy_(b)
                mod._buffers[name] = v
                off += b.numel()
            self.flats.append(flat)
        self.bytes = sum(f.numel() * f.element_size() for f in self.flats)

    def __call__(self):
        for f in self.flats:
            dist.broadcast(f, 0, group=self.group)


class TrainStep:
    def __init__(self, model, forward_loss, optimizer, graph=True, warmup=3, group=None, bucket_mb=32,
                 accum_steps=1, overlap=True, force_collectives=False, grad_comm_dtype=None, early_params=None):
        """``force_collectives``: issue the bucket all-reduces and the buffer broadcast even in
        a world of one (test switch; needs an initialised process group).  A failure to
        capture the collectives raises, unless EWVIT_GRAPH_SPLIT_FALLBACK=1 allows the split,
        non-overlapped form (graphs around one all-reduce) — never silently.
        ``grad_comm_dtype``: None / torch.float32 (default, the reference's fp32 gradient) or
        torch.bfloat16 — the buckets all-reduced in bf16 (GradBuckets; default from
        EWVIT_GRAD_COMM_DTYPE=bf16)."""
        if grad_comm_dtype is None and os.environ.get('EWVIT_GRAD_COMM_DTYPE', 'fp32').lower() in ('bf16', 'bfloat16'):
            grad_comm_dtype = torch.bfloat16
        self.model, self.forward_loss, self.opt, self.group = model, forward_loss, optimizer, group
        self.world = _world(group)
        forced = bool(force_collectives) and dist.is_available() and dist.is_initialized()
        if force_collectives and not forced:
            raise RuntimeError('TrainStep(force_collectives=True) needs an initialised process group')
        self.accum = int(accum_steps)
        self.params = [p for p in model.parameters() if p.requires_grad]
        dev = self.params[0].device
        backend = dist.get_backend(group) if (self.world > 1 or forced) else None
        capturable = backend in (None, 'nccl')
        self.graph = bool(graph) and dev.type == 'cuda' and capturable
        dp = self.world > 1 or forced
        self.buckets = GradBuckets(self.params, group, bucket_mb, force=forced, comm_dtype=grad_comm_dtype) if dp else None
        if self.buckets is not None:
            self.buckets.defer = not overlap
        self.bufsync = BufferSync(model, group) if dp else None
        self._early_init(early_params)
        self.loss = None
        self.mode = 'graph' if self.graph else 'eager'
        self._hyper = optimizer.hyper_signature() if hasattr(optimizer, 'hyper_signature') else None
        self._started = False
        self.g2 = None
        self.fallback = None
        self._capturing = False
        self._capture_mode = os.environ.get('EWVIT_CAPTURE_MODE', 'relaxed')
        if self.graph and self.buckets is not None and self.buckets.defer:
            self._capture_split(warmup)
        elif self.graph:
            try:
                self._capture(warmup)
            except Exception as e:          # noqa: BLE001 — a backend that cannot record collectives
                self.g = None                # a failed capture's graph is never replayed
                if self.buckets is None or os.environ.get('EWVIT_GRAPH_SPLIT_FALLBACK', '0') != '1':
                    import sys
                    import traceback
                    print('TrainStep: graph capture failed:', file=sys.stderr)
                    traceback.print_exc()
                    sys.stderr.flush()
                    self.close()             # no gradient hooks / slots left behind on the parameters
                    raise
                import sys
                print(f'TrainStep: capturing the collectives failed ({type(e).__name__}: {e}); '
                      f'EWVIT_GRAPH_SPLIT_FALLBACK=1: forward/backward and optimizer graphs around one '
                      f'all-reduce', file=sys.stderr, flush=True)
                torch.cuda.synchronize()
                self.buckets.defer = True
                self.fallback = f'{type(e).__name__}: {e}'
                self._capture_split(warmup)

    # ---- early optimizer step: the parameters whose gradients are final long before the end of
    # the backward pass (DAMA: everything but the backbone, whose backward is the critical path)
    # are updated on a side stream as soon as the last of their gradients has been accumulated,
    # so only the backbone's update remains after the backward pass.  Per-parameter Adam: the
    # same bits as one step() (tests/test_gpu_graph.py).  World 1, one micro-batch, an optimizer
    # with step_subset (ewvit.optim.Adam); their weight gradients are never deferred
    # (ewvit.grads.deferrable), so the last accumulation is the last write.  Opt-in
    # (EWVIT_EARLY_STEP=1): at config 2 the early update's 1.1 GB of HBM traffic beside the two
    # branches costs more than the ~190 us it takes off the end of the step (3833-3838 against
    # 3888-3891 frames/s, profiles/r06/s2/ab/early_step.log).
    def _early_init(self, early_params):
        self._early = None
        if (early_params is None or os.environ.get('EWVIT_EARLY_STEP', '0') != '1' or self.world > 1
                or self.accum != 1 or not hasattr(self.opt, 'step_subset')):
            return
        train = {id(p) for p in self.params}
        early = [p for p in early_params if id(p) in train]
        if not early or len(early) == len(self.params):
            return
        eids = {id(p) for p in early}
        self._early = {'ids': eids, 'late': {id(p) for p in self.params if id(p) not in eids}, 'n': len(early),
                       'left': 0, 'events': {}, 'fired': False, 'on': False, 'stream': None}
        for p in early:
            p._ewvit_early = True
        self._early['hooks'] = [p.register_post_accumulate_grad_hook(self._early_hook) for p in early]
        self.opt._split_steps = 2

    def _early_hook(self, p):
        e = self._early
        if e is None or not e['on'] or p.grad is None:
            return
        if p.grad.is_cuda:
            st = torch.cuda.current_stream(p.grad.device)
            ev = torch.cuda.Event()
            ev.record(st)
            e['events'][st.cuda_stream] = ev         # the stream's latest gradient write
        e['left'] -= 1
        if e['left'] == 0:
            if e['stream'] is None:
                e['stream'] = torch.cuda.Stream(device=p.device)
            side = e['stream']
            for ev in e['events'].values():
                side.wait_event(ev)
            with torch.cuda.stream(side):
                self.opt.step_subset('early', e['ids'])
            e['fired'] = True

    def _early_close(self):
        e = getattr(self, '_early', None)
        if e is None:
            return
        for h in e['hooks']:
            h.remove()
        for p in self.params:
            if id(p) in e['ids'] and hasattr(p, '_ewvit_early'):
                del p._ewvit_early
        self.opt.__dict__.pop('_split_steps', None)
        self._early = None

    def _opt_step(self):
        e = self._early
        if e is None:
            self.opt.step()
            return
        e['on'] = False
        if e['fired']:
            torch.cuda.current_stream().wait_stream(e['stream'])
            self.opt.step_subset('late', e['late'])
        else:                                        # not every early gradient arrived: one step
            self.opt.step_subset('early', e['ids'])
            self.opt.step_subset('late', e['late'])

    def close(self):
        """Release the captured graphs (after the device has drained them) and detach from the
        model: remove the gradient hooks and slots of the buckets.  Call it while the process
        group is still alive — a graph holding RCCL collectives releases communicator
        resources when it is destroyed — before ``destroy_process_group``."""
        if getattr(self, 'g', None) is not None or getattr(self, 'g2', None) is not None:
            torch.cuda.synchronize()
            for name in ('g', 'g2'):
                gr = getattr(self, name, None)
                if gr is not None:
                    gr.reset()
                    setattr(self, name, None)
            torch.cuda.synchronize()
            rel = getattr(self.opt, 'release_capture', None)
            if rel is not None:
                rel()                        # (the optimizer no longer guards released graphs' state)
        if self.buckets is not None:
            self.buckets.remove()
            self.buckets = None
        self._early_close()

    def describe(self):
        d = {'launch': 'hip-graph' if self.graph else 'eager', 'world': self.world}
        if self.fallback is not None:
            d['capture_fallback'] = self.fallback
        if self.buckets is not None:
            d.update({'buckets': len(self.buckets.buckets), 'bucket_mb': self.buckets.bucket_bytes / (1 << 20),
                      'grad_bytes': 4 * self.buckets.flat.numel(), 'buffer_bytes': self.bufsync.bytes,
                      'overlap': 'per-bucket all-reduce issued during backward' + (
                          ', recorded in the step graph' if self.graph else '')
                      if not self.buckets.defer else 'one all-reduce between two graphs'})
        return d

    def _first(self):
        self._eager()                        # first step: observes the gradient order
        if self.buckets is not None:
            self.buckets.relayout()
        self._started = True
        return self.loss

    # ---- one iteration
    def _fwd_bwd(self):
        from . import conv
        loss = None
        with conv.packed():          # every conv weight packed to bf16 by one launch
            for k in range(self.accum):
                if self.buckets is not None:
                    self.buckets.collect = k == self.accum - 1
                grads.begin_step()           # parameter use counts (ewvit.grads)
                try:
                    lk = self.forward_loss(k) if self.accum > 1 else self.forward_loss()
                    if self.accum > 1:
                        lk = lk / self.accum                               # train.py:110
                    lk.backward()
                finally:
                    grads.end_step()
                loss = lk.detach() if loss is None else loss + lk.detach()
        return loss

    def _iteration(self):
        self.opt.zero_grad(set_to_none=True)
        if self.buckets is not None:
            self.bufsync()
            self.buckets.begin()
        if self._early is not None:
            self._early.update(left=self._early['n'], events={}, fired=False, on=True)
        loss = self._fwd_bwd()
        if self.buckets is not None:
            self.buckets.finish()
        self._opt_step()
        return loss

    def _eager(self):
        self.loss = self._split_eager() if (self.buckets is not None and self.buckets.defer) else self._iteration()
        return self.loss

    # ---- capture: warm-up and capture on one side stream (the AccumulateGrad nodes keep
    # the stream they were created on), no autograd graph kept alive across them
    def _capture(self, warmup):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._first()
            for _ in range(max(0, warmup - 1)):       # lazy inits (library handles, caches, RCCL comms)
                self._iteration()
            self.loss = None
            torch.cuda.synchronize()
            self._drain_watchdog()
            self.g = torch.cuda.CUDAGraph()
            # the host seeds the recorded dropout launches bake in come from the CPU generator
            # (ewvit.ops._seed); its state at capture lets a caller reproduce a replay eagerly
            self.capture_cpu_rng = torch.get_rng_state()
            # relaxed capture: CUDA calls of other threads — the process group's watchdog
            # polling the events of the eager collectives that preceded the capture, a
            # data-loader thread — must neither fail nor invalidate the capture.  In the
            # default global mode the watchdog's event query errors and it aborts the process
            # (seen intermittently on the GPU box; TORCH_NCCL_ASYNC_ERROR_HANDLING=0 hides it)
            self._capturing = True
            try:
                with torch.cuda.graph(self.g, stream=side, capture_error_mode=self._capture_mode):
                    self.loss = self._iteration()
            finally:
                self._capturing = False      # the capture has ended (the context closed it)
            self._finish_capture(self.g)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()

    def _capture_split(self, warmup):
        """Fallback: g1 = forward + backward (+ gradient slots), the all-reduce issued
        eagerly, g2 = optimizer."""
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self._split_eager()
            self.loss = None
            torch.cuda.synchronize()
            self._drain_watchdog()
            self.opt.zero_grad(set_to_none=True)
            self.g = torch.cuda.CUDAGraph()
            self._capturing = True
            try:
                with torch.cuda.graph(self.g, stream=side, capture_error_mode=self._capture_mode):
                    self.buckets.begin()
                    self.loss = self._fwd_bwd()
                    self.buckets.finish()
                self.g2 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g2, stream=side, pool=self.g.pool(), capture_error_mode=self._capture_mode):
                    self.opt.step()
            finally:
                self._capturing = False
            self._finish_capture(self.g2)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()

    def _drain_watchdog(self):
        """Before a capture that records RCCL collectives.  Every EAGER collective (the warm-up
        steps' bucket all-reduces and buffer broadcasts, the layout broadcast) is queued to
        ProcessGroupNCCL's watchdog thread, which polls the collective's end event
        (hipEventQuery) until it sees it complete and then drops it (about every 100 ms:
        tools/fr_probe.py, profiles/r04/fr_probe.log).  Those events were recorded on the
        process group's stream, and the first collective of the capture makes that stream
        part of the capture: a poll of such an event from the watchdog thread while the capture
        runs fails with hipErrorCapturedEvent ("operation not permitted on an event last
        recorded in a capturing stream") in EITHER capture mode — the watchdog rethrows and
        aborts the process, and the capture itself is invalidated (the next launch of the
        capturing thread reports "operation failed due to a previous error during capture";
        profiles/r04/dp_abort.log).  So, in both modes: after the device has drained, wait until
        the watchdog has retired every collective enqueued so far — its own progress marker,
        `last_completed_collective == last_enqueued_collective` of each process group in the
        flight-recorder status (TORCH_FR_BUFFER_SIZE > 0 before the group is created:
        ewvit.dist.rccl_env) — so its queue is empty when the capture begins.  Collectives issued
        during the capture are never queued."""
        if not (self.buckets is not None and self.buckets.reduce and dist.get_backend(self.group) == 'nccl'):
            return
        # Both preconditions are hard errors (verdict r4): either one missing brings the round-3
        # watchdog abort back, later and in another thread.  EWVIT_ALLOW_UNDRAINED_CAPTURE=1
        # turns them into warnings (a torch build without the flight recorder, at the caller's risk).
        unsafe = os.environ.get('EWVIT_ALLOW_UNDRAINED_CAPTURE', '0') == '1'

        def refuse(msg):
            if not unsafe:
                raise RuntimeError(msg + ' (EWVIT_ALLOW_UNDRAINED_CAPTURE=1 to capture anyway)')
            import warnings
            warnings.warn(msg)

        if os.environ.get('TORCH_NCCL_CUDA_EVENT_CACHE', '1') != '0':
            refuse('TrainStep: refusing to capture RCCL collectives with the process group\'s CUDA event cache '
                   'on: a later eager collective can reuse a captured event and abort the NCCL watchdog '
                   '(hipErrorCapturedEvent); call ewvit.dist.rccl_env() (or set TORCH_NCCL_CUDA_EVENT_CACHE=0) '
                   'before init_process_group')
        if not _pg_status():
            refuse('TrainStep: refusing to capture RCCL collectives: the flight recorder\'s process-group status '
                   'is unavailable (TORCH_FR_BUFFER_SIZE unset before init_process_group, or this torch build '
                   'has no _dump_nccl_trace_json), so the NCCL watchdog queue cannot be drained before the '
                   'capture; call ewvit.dist.rccl_env() before init_process_group')
            return
        retire_eager_collectives()

    def _finish_capture(self, graph):
        fin = getattr(self.opt, 'finish_capture', None)
        if fin is not None:
            fin(graph)                       # device tables the captured optimizer launches read,
        torch.cuda.synchronize()             # owned by the graph that reads them

    def _split_eager(self):
        self.opt.zero_grad(set_to_none=True)
        self.bufsync()
        self.buckets.begin()
        loss = self._fwd_bwd()
        self.buckets.finish()
        self.buckets.allreduce_all()
        self.opt.step()
        return loss

    def __call__(self):
        """One training iteration; returns the (static, detached) loss tensor."""
        if not self.graph:
            return self._eager() if self._started else self._first()
        if self._hyper is not None and self.opt.hyper_signature() != self._hyper:
            raise RuntimeError('TrainStep: betas / eps / weight_decay changed after capture; build a new TrainStep')
        if hasattr(self.opt, 'sync_hyper'):
            self.opt.sync_hyper()            # LR schedule -> the device scalar the graph reads
        if self.g2 is not None:
            self.bufsync()
            self.g.replay()
            self.buckets.allreduce_all()
            self.g2.replay()
            return self.loss
        self.g.replay()
        return self.loss
