"""Time the stem direct conv (ewvit_conv2d_stem_fwd, config-2 shape: 64 frames x 3 x 224^2
fp32 -> 64 x 112^2 x 24 bf16 + BN partials) over back-to-back launches; EWVIT_STEM_GRID
picks the workgroup count (A/B)."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'efficient-wavelet-vit_amd')]
import ewvit  # noqa: E402

x = torch.randn(64, 3, 224, 224, device='cuda')
w = (torch.randn(24, 3, 3, 3, device='cuda') / 5).contiguous(memory_format=torch.channels_last)
sh = torch.zeros(24, device='cuda')
for stats in (True, False):
    for _ in range(3):
        ewvit.conv.stem_conv2d(x, w, None, 2, sh, stats=stats)
    torch.cuda.synchronize()
    # replayed from a HIP graph: the per-call host work (ctypes, allocations) is not timed
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
        for _ in range(20):
            ewvit.conv.stem_conv2d(x, w, None, 2, sh, stats=stats)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 100 * 1e3
    print(f"grid={os.environ.get('EWVIT_STEM_GRID', 'default')} stats={stats}: {us:.1f} us per call "
          f"(incl. weight copy{' + fold' if stats else ''}), {77.07e6 / us / 1e6:.2f} TB/s")
