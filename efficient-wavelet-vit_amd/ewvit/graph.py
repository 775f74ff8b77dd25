"""A static-shape data-parallel training step, replayed from captured HIP graphs.

The reference's training iteration (train.py:93-115: DeepfakeDetector forward over
the chunk, combined_loss, backward, optimizer step) issues ~2000 kernel launches;
issued from Python each costs 10-50 us of host time, which is more than the GPU
needs for most of them.  `TrainStep` records the iteration once into HIP graphs
(torch.cuda.CUDAGraph is hipGraph on ROCm) and replays it: one host call per step.

Data parallel (one process per GPU): the gradient all-reduce runs between two
graphs — g1 = forward + loss + backward + pack of all gradients into ONE flat fp32
buffer; then a single RCCL all-reduce of that buffer over xGMI; g2 = average +
optimizer step reading the gradients as views of the flat buffer.  Before g1 the
module buffers (BatchNorm running statistics and counters) are broadcast from
rank 0, which is what DistributedDataParallel(broadcast_buffers=True) does and what
the reference's nn.DataParallel replicas see (train.py:136-139).  `graph=False`
runs the identical sequence eagerly (the path the CPU gloo tests drive).

Requirements of graph mode: every input of `forward_loss` is a static tensor
updated in place, the model issues no host synchronisation, and random draws use
the device generator (torch ops) or the ewvit dropout step counter
(_lib.rng_advance, advanced inside the recorded forward).
"""
import torch
import torch.distributed as dist


def _world(group):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


class TrainStep:
    def __init__(self, model, forward_loss, optimizer, graph=True, warmup=3, group=None):
        self.model, self.forward_loss, self.opt, self.group = model, forward_loss, optimizer, group
        self.world = _world(group)
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.buffers = [b for b in model.buffers()]
        dev = self.params[0].device
        self.graph = bool(graph) and dev.type == 'cuda'
        self.flat = None
        if self.world > 1:
            n = sum(p.numel() for p in self.params)
            self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
            self.views, off = [], 0
            for p in self.params:
                # the parameter's own strides (channels-last conv weights included), so
                # the fused optimizer pairs gradient and parameter memory element-wise
                self.views.append(self.flat.as_strided(p.shape, p.stride(), off))
                off += p.numel()
        self.loss = None
        if self.graph:
            self._capture(warmup)

    # ---- pieces of one iteration
    def _sync_buffers(self):
        if self.world > 1 and self.buffers:
            dist._broadcast_coalesced(self.group or dist.group.WORLD, self.buffers, 64 << 20, 0)

    def _fwd_bwd(self):
        from . import conv
        with conv.packed():          # every conv weight packed to bf16 by one launch
            loss = self.forward_loss()
            loss.backward()
        if self.world > 1:
            torch._foreach_copy_(self.views, [p.grad for p in self.params])
        return loss

    def _allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.flat, group=self.group)

    def _update(self):
        if self.world > 1:
            self.flat.div_(self.world)
        self.opt.step()

    def _eager(self):
        self.opt.zero_grad(set_to_none=True)
        self._sync_buffers()
        loss = self._fwd_bwd()
        self._allreduce()
        if self.world > 1:
            for p, v in zip(self.params, self.views):
                p.grad = v
        self._update()
        return loss

    # ---- capture
    def _capture(self, warmup):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):          # lazy inits (library handles, caches) happen here
                self._eager()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.opt.zero_grad(set_to_none=True)
        self._sync_buffers()
        self.g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g1):
            self.loss = self._fwd_bwd()
            if self.world == 1:
                self._update()
        self.g2 = None
        if self.world > 1:
            for p, v in zip(self.params, self.views):
                p.grad = v
            self.g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g2, pool=self.g1.pool()):
                self._update()
        torch.cuda.synchronize()

    def __call__(self):
        """One training iteration; returns the (static) loss tensor."""
        if not self.graph:
            self.loss = self._eager()
            return self.loss
        self._sync_buffers()
        self.g1.replay()
        if self.g2 is not None:
            self._allreduce()
            self.g2.replay()
        return self.loss
