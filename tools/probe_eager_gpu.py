"""Probe: the reference's op sequence in torch eager on one MI355X (the oracle
restatement moved to cuda), bf16 autocast, 64-frame chunk, fwd+bwd+Adam.
Prints frames/s and the top GPU kernels (torch.profiler).  Measurement aid for
DESIGN.md — the "what PyTorch eager does with the reference code" baseline."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import model as om  # noqa: E402


def main():
    frames = int(os.environ.get('FRAMES', 64))
    cl = os.environ.get('CL', '1') == '1'
    dev = 'cuda'
    torch.manual_seed(0)
    m = om.DeepfakeDetector(3, 128, batch_size=frames).to(dev)
    if cl:
        m = m.to(memory_format=torch.channels_last)
    opt = torch.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=1e-4, weight_decay=1e-4)
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5], device=dev))
    x = torch.randn(8, frames // 8, 3, 224, 224, device=dev)
    if cl:
        x = x.contiguous()
    y = torch.bernoulli(torch.full((8,), 0.5, device=dev))

    def step():
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = m(x, frames // 8, 'dynamic')
        loss = om.combined_loss({k: v.float() for k, v in out.items()}, y, crit, 1, 1)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    n = 10
    t = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / n
    print(f'EAGER bf16-autocast channels_last={cl}: {dt*1e3:.2f} ms/step, {frames/dt:.1f} frames/s', flush=True)
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by='cuda_time_total', row_limit=45, max_name_column_width=90))


if __name__ == '__main__':
    main()
