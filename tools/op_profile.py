"""Attribute GPU time of the bench step to torch ops with input shapes
(torch.profiler, record_shapes) — measurement aid for choosing the next kernel."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))

import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    step = bench.build_step(dev, 64, 0)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by='cuda_time_total', row_limit=70, max_name_column_width=40, max_shapes_column_width=110))


if __name__ == '__main__':
    main()
