"""One DAMA branch (forward + backward) replayed from its own HIP graph N times — a target for
`rocprofv3 --kernel-trace --stats` (kernel durations and the gaps between them without the
other branch or the per-launch events of bench.py's eager pass).

  python tools/piece_trace.py [--piece sfe|mwt] [--reps 5]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))
sys.path.insert(0, os.path.join(REPO, 'tools'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--piece', default='sfe', choices=('sfe', 'mwt'))
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    import bench
    from branch_time import _NoOpt
    from ewvit.graph import TrainStep
    dev = torch.device('cuda', 0)
    full = bench.build_step(dev, 64, 0, graph=True, config=2)
    full.close()
    model = full.model
    x = torch.randn(64, 3, 224, 224, device=dev)
    mod = getattr(model.dama, args.piece)

    def fl():
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y = mod(x)
        return y.float().square().mean()
    st = TrainStep(model, fl, _NoOpt(model.parameters()), graph=True)
    torch.cuda.synchronize()
    torch.cuda.nvtx.range_push('replays') if hasattr(torch.cuda, 'nvtx') else None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        st()
    e1.record()
    torch.cuda.synchronize()
    print(f'{args.piece}: {e0.elapsed_time(e1) / args.reps:.3f} ms per replay', flush=True)


if __name__ == '__main__':
    main()
