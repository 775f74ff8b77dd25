"""Which branch bounds the config-2 step: each piece of the DAMA training step (forward +
backward, no optimizer) replayed alone from a HIP graph, timed with events over N replays.

  mwt        the MWT branch alone, on the whole chip (uncapped)
  mwt_cap    the MWT branch alone under the grid cap the step runs it with (EWVIT_MWT_GRID_CAP)
  sfe        the SFE branch (EfficientNetV2-S backbone + ViT head) alone
  full       the whole DeepfakeDetector forward + combined_loss + backward (both streams)
  step       `full` + Adam (the bench's TrainStep)

Usage: python tools/branch_time.py [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


class _NoOpt:
    """No update; zero_grad drops the gradients like the real optimizer (else every replay
    would add into .grad: ~480 accumulation kernels in the SFE piece)."""

    def __init__(self, params=()):
        self.params = list(params)

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def step(self):
        pass


def _time(step, reps):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        step()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--tables', type=int, default=0, help='also print per-entry tables (N top launch configs)')
    args = ap.parse_args()
    import bench
    import ewvit
    from ewvit.graph import TrainStep
    from network.dama import _mwt_grid_cap
    dev = torch.device('cuda', 0)
    full = bench.build_step(dev, 64, 0, graph=True, config=2)
    model = full.model
    x = torch.randn(64, 3, 224, 224, device=dev)
    out = {'step_ms': _time(full, args.reps)}
    for p in model.parameters():
        p.grad = None

    def piece(fn):
        def fl():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                y = fn()
            return y.float().square().mean()
        return TrainStep(model, fl, _NoOpt(model.parameters()), graph=True)
    dama = model.dama
    out['mwt_ms'] = _time(piece(lambda: dama.mwt(x)), args.reps)
    cap = _mwt_grid_cap()

    def mwt_capped():
        with ewvit._lib.grid_cap(cap):
            return dama.mwt(x)
    out['mwt_cap_ms'] = _time(piece(mwt_capped), args.reps)
    out['mwt_cap'] = cap
    out['sfe_ms'] = _time(piece(lambda: dama.sfe(x)), args.reps)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
    if args.tables:
        # per-entry event timings of each piece issued eagerly, one stream, uncapped
        for name, fn in (('mwt', lambda: dama.mwt(x)), ('sfe', lambda: dama.sfe(x))):
            st = piece(fn)
            ewvit._lib.enable_timing(True)
            for _ in range(3):
                st._eager()
            torch.cuda.synchronize()
            tab = bench.kernel_table(ewvit._lib.timing_records())
            shapes = bench.shape_table(ewvit._lib.timing_detail())
            ewvit._lib.enable_timing(False)
            tot = sum(v['total_ms'] for v in tab.values()) / 3
            print(f'--- {name}: {tot:.3f} ms of kernel time per pass, '
                  f'{sum(v["launches"] for v in tab.values()) / 3:.0f} launches')
            for k, v in sorted(tab.items(), key=lambda kv: -kv[1]['total_ms'])[:25]:
                print(f"{k:36s} {v['launches'] / 3:5.0f} {v['total_ms'] / 3:7.3f} ms {v['avg_us']:7.1f} us "
                      f"{v['TFLOP/s']:7.1f} TF/s {v['GB/s']:7.0f} GB/s")
            print(f'top launch configurations ({name}):')
            for r in shapes[:args.tables]:
                print(f"  {r['entry']:34s} {str(r['args'])[:70]:70s} x{r['launches'] / 3:3.0f} "
                      f"{r['total_ms'] / 3:7.3f} ms {r['avg_us']:7.1f} us {r['TFLOP/s']:6.1f} TF/s {r['GB/s']:6.0f} GB/s")


if __name__ == '__main__':
    main()
