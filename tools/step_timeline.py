"""Device timeline of one replayed config-2 step, from wall-clock probes the step records as
its streams reach marked points (EWVIT_PROBE=1, ewvit/probe.py) — no profiler in the loop, so
the branches overlap as they do in the bench.  Milliseconds since the fork (slot 0):

  1 SFE forward end (main)          2 MWT forward start (side)     3 MWT forward end (side)
  4 SFE backward start (main)       5 MWT backward start (side)       9 step end (after Adam)
  7 backbone forward end (main)     6 token-path backward end = backbone backward start (main)
  8 last MWT parameter gradient accumulated (~ MWT backward end)
 10 last SFE parameter gradient accumulated (~ backbone backward end)

Usage: python tools/step_timeline.py [--steps 5]  (sets EWVIT_PROBE=1 itself)"""
import argparse
import json
import os
import sys

os.environ['EWVIT_PROBE'] = '1'
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=5)
    a = ap.parse_args()
    import bench
    import ewvit
    from ewvit import dist as edist, probe
    edist.rccl_env()
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    edist.init_from_env('nccl')
    ewvit.load_library()
    probe.buffer(dev)                       # allocated before any capture
    step = bench.build_step(dev, bench.CONFIGS[2]['frames'], 0, graph=True, config=2)
    rows = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        step()
        probe.stamp(9, dev)
        torch.cuda.synchronize()
        rows.append(probe.read(dev))
    med = {k: round(sorted(r[k] for r in rows)[len(rows) // 2], 3) for k in rows[-1]}
    print(json.dumps({'env': {k: v for k, v in os.environ.items() if k.startswith('EWVIT_')}, 'ms': med}), flush=True)
    if hasattr(step, 'close'):
        step.close()


if __name__ == '__main__':
    main()
