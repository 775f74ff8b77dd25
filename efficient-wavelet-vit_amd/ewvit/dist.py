"""Multi-GPU data parallelism for the training step (replaces the reference's
``nn.DataParallel`` at train.py:249-251).

One process per GPU (torchrun / torch.distributed.run), ``DistributedDataParallel``
over RCCL (backend 'nccl' on ROCm) with gradient all-reduce bucketed and overlapped
with backward.  Semantics kept from the reference's DataParallel:

* videos (dim 0 of [B, K, 3, H, W]) are split over ranks and each rank runs its own
  frame chunks — BatchNorm batch statistics and the ``pos_embedding[0:N]`` chunk
  position are per replica, exactly as DataParallel's per-replica forward;
* ``broadcast_buffers=True``: rank 0's BatchNorm running statistics are broadcast at
  every forward, as DataParallel re-replicates device 0's buffers every call;
* gradients are averaged over ranks (DataParallel sums per-replica grads of a loss
  that is a mean over the full batch: same value when every rank holds B/world videos).

Structurally unused parameters (the ablation heads, ``sfe.mlp_head``) are frozen by
``DeepfakeDetector`` so DDP needs no ``find_unused_parameters`` scan.
"""
import os

import torch
import torch.distributed as dist


def env_ranks():
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', str(rank)))
    return rank, world, local


def rccl_env():
    """Process-group settings the captured step needs; they are read when a ProcessGroupNCCL
    is constructed, so call this before ``init_process_group``.

    * ``TORCH_NCCL_CUDA_EVENT_CACHE=0``: the end event of every collective is a fresh
      event.  With the cache on, the events of collectives recorded inside a HIP graph
      capture go back to the cache when their Work objects die, and a later EAGER collective
      can be handed one of them; ProcessGroupNCCL's watchdog thread then queries it and HIP
      answers hipErrorCapturedEvent ("operation not permitted on an event last recorded in a
      capturing stream") — the watchdog rethrows and the process aborts.  Seen on the GPU box
      as soon as a process issues eager collectives after a captured step (a second
      TrainStep, the bench's eager timing pass): profiles/r04/dp_abort.log.
    * ``TORCH_FR_BUFFER_SIZE``: the flight recorder's process-group status, which a
      global-mode capture waits on (ewvit.graph.retire_eager_collectives).
    * ``TORCH_NCCL_AVOID_RECORD_STREAMS``: the gradient buckets are persistent buffers."""
    os.environ.setdefault('TORCH_NCCL_CUDA_EVENT_CACHE', '0')
    os.environ.setdefault('TORCH_FR_BUFFER_SIZE', '2000')
    os.environ.setdefault('TORCH_NCCL_AVOID_RECORD_STREAMS', '1')


def init_from_env(backend=None):
    """Initialise the process group from torchrun's env (MASTER_ADDR/PORT).
    backend: 'nccl' (RCCL) when a GPU is used, 'gloo' otherwise."""
    rank, world, local = env_ranks()
    rccl_env()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = 'nccl' if torch.cuda.is_available() else 'gloo'
        dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world, local


def wrap(model, device=None, bucket_cap_mb=64):
    """DDP-wrap `model` when a multi-rank group is up; identity otherwise.
    64 MB buckets: the ~60 M trainable fp32 params (240 MB of grads) go in ~4
    all-reduces, each large enough to run at link bandwidth on xGMI."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return model
    ids = [device.index] if device is not None and device.type == 'cuda' else None
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=ids, broadcast_buffers=True,
                                                     gradient_as_bucket_view=True, bucket_cap_mb=bucket_cap_mb)


def shard_videos(x, rank, world):
    """The videos of a global batch [B, K, ...] that rank `rank` processes."""
    B = x.shape[0]
    per = (B + world - 1) // world
    return x[rank * per:min(B, (rank + 1) * per)]


def rank_generator(base_seed, rank, device='cpu'):
    return torch.Generator(device=device).manual_seed(base_seed + rank)


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (the bench's timing rule)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
