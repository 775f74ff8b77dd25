"""Host side of the replayed step: how long step() takes to RETURN (the HIP graph launch:
host-side packet submission of every node) against the whole step (launch + device time), per
step, over --steps replays of the bench's config-2 TrainStep.  A launch time close to the step
time means the device waits on the host's submission, not on its kernels.

Usage: python tools/graph_launch.py [--config 2] [--steps 10]"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--frames', type=int, default=None)
    a = ap.parse_args()
    import bench
    import ewvit
    from ewvit import dist as edist
    edist.rccl_env()
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    edist.init_from_env('nccl')
    ewvit.load_library()
    frames = a.frames or (32 if a.config == 4 else bench.CONFIGS[a.config]['frames'])
    step = bench.build_step(dev, frames, 0, graph=True, config=a.config)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    launch, total = [], []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        launch.append((t1 - t0) * 1e3)
        total.append((t2 - t0) * 1e3)
    # back to back (the bench's loop): the next launch overlaps the previous step's tail
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    b2b = (time.perf_counter() - t0) * 1e3 / a.steps
    env = {k: os.environ[k] for k in os.environ if k.startswith(('DEBUG_HIP', 'DEBUG_CLR', 'EWVIT_', 'GPU_MAX'))}
    print(json.dumps({'config': a.config, 'frames': frames, 'env': env,
                      'launch_ms': sorted(launch)[len(launch) // 2], 'step_ms': sorted(total)[len(total) // 2],
                      'back_to_back_ms': round(b2b, 3)}), flush=True)
    if hasattr(step, 'close'):
        step.close()


if __name__ == '__main__':
    main()
